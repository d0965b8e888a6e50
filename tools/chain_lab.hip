// chain_lab.hip — cost per entry of the stored-order fp64 chain s -= p[k] over LDS (lab only).
//
// The exact GS-CF engines (sss_gs_persist.hip) end every row with one lane subtracting the row's
// staged products from b_i in stored order: a dependent fp64 chain over LDS.  This lab times, in
// one wave, the chain over 2048 LDS products for several read schedules (cycles per entry from
// s_memtime), and checks every schedule gives the same bits.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/chain_lab.hip -o tools/chain_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

constexpr int M = 2048;

// the engine's schedule: 8 reads ahead of 8 dependent subtractions
__device__ double chain8(double s, const double *p, int a, int e)
{
    int k = a;
    if (e - k >= 16) {
        double c0 = p[k], c1 = p[k + 1], c2 = p[k + 2], c3 = p[k + 3];
        double c4 = p[k + 4], c5 = p[k + 5], c6 = p[k + 6], c7 = p[k + 7];
        for (k += 8; k + 8 <= e; k += 8) {
            const double n0 = p[k], n1 = p[k + 1], n2 = p[k + 2], n3 = p[k + 3];
            const double n4 = p[k + 4], n5 = p[k + 5], n6 = p[k + 6], n7 = p[k + 7];
            s -= c0; s -= c1; s -= c2; s -= c3; s -= c4; s -= c5; s -= c6; s -= c7;
            c0 = n0, c1 = n1, c2 = n2, c3 = n3, c4 = n4, c5 = n5, c6 = n6, c7 = n7;
        }
        s -= c0; s -= c1; s -= c2; s -= c3; s -= c4; s -= c5; s -= c6; s -= c7;
    }
    for (; k < e; ++k) s -= p[k];
    return s;
}
// 16 ahead, read as 16-byte pairs
__device__ double chain16(double s, const double *p, int a, int e)
{
    int k = a;
    if ((k & 1) && k < e) s -= p[k++];   // 16-byte alignment of the pair reads
    if (e - k >= 32) {
        double2 c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = *reinterpret_cast<const double2 *>(p + k + 2 * u);
        for (k += 16; k + 16 <= e; k += 16) {
            double2 n[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) n[u] = *reinterpret_cast<const double2 *>(p + k + 2 * u);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s -= c[u].x;
                s -= c[u].y;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) c[u] = n[u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            s -= c[u].x;
            s -= c[u].y;
        }
    }
    for (; k < e; ++k) s -= p[k];
    return s;
}
// the chain from registers only (the floor: dependent subtractions alone)
__device__ double chain_reg(double s, const double *p, int a, int e)
{
    double r[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) r[u] = p[u];
    for (int k = a; k + 16 <= e; k += 16)
#pragma unroll
        for (int u = 0; u < 16; ++u) s -= r[u];
    return s;
}

template <int V>
__global__ __launch_bounds__(64) void kchain(const double *src, double *out, long long *cyc, int m)
{
    __shared__ double p[M];
    for (int t = threadIdx.x; t < M; t += 64) p[t] = src[t];
    __syncthreads();
    double s = 1.0;
    long long t0 = 0, t1 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        if (V == 0) s = chain8(s, p, 0, m);
        else if (V == 1) s = chain16(s, p, 0, m);
        else s = chain_reg(s, p, 0, m);
        out[0] = s;
        t1 = __builtin_amdgcn_s_memtime();
        cyc[0] = t1 - t0;
    }
}

int main()
{
    double h[M];
    for (int i = 0; i < M; ++i) h[i] = 1e-3 * ((i * 7919) % 1013) - 0.5;
    double *src, *out;
    long long *cyc;
    CK(hipMalloc(&src, sizeof h));
    CK(hipMalloc(&out, 8));
    CK(hipMalloc(&cyc, 8));
    CK(hipMemcpy(src, h, sizeof h, hipMemcpyHostToDevice));
    const char *names[3] = {"8 ahead (engine)", "16 ahead, 16-B reads", "registers (floor)"};
    double ref = 0;
    for (int v = 0; v < 3; ++v) {
        long long best = 1LL << 60;
        double s = 0;
        for (int rep = 0; rep < 5; ++rep) {
            if (v == 0) hipLaunchKernelGGL(kchain<0>, dim3(1), dim3(64), 0, 0, src, out, cyc, M);
            if (v == 1) hipLaunchKernelGGL(kchain<1>, dim3(1), dim3(64), 0, 0, src, out, cyc, M);
            if (v == 2) hipLaunchKernelGGL(kchain<2>, dim3(1), dim3(64), 0, 0, src, out, cyc, M);
            CK(hipDeviceSynchronize());
            long long c;
            CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&s, out, 8, hipMemcpyDeviceToHost));
            if (c < best) best = c;
        }
        if (v == 0) ref = s;
        printf("%-24s %8lld s_memtime ticks for %d entries (%.2f per entry)%s\n", names[v], best, M, (double)best / M,
               v < 2 ? (memcmp(&s, &ref, 8) ? "  MISMATCH" : "  bitwise ok") : "");
    }
    return 0;
}
