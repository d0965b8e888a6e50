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
// 16 ahead, two register sets in turn (no copies between them)
__device__ double chain_pp(double s, const double *p, int a, int e)
{
    int k = a;
    if ((k & 1) && k < e) s -= p[k++];
    if (e - k >= 32) {
        double2 c[8], d[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = *reinterpret_cast<const double2 *>(p + k + 2 * u);
        for (; k + 32 <= e; k += 32) {
#pragma unroll
            for (int u = 0; u < 8; ++u) d[u] = *reinterpret_cast<const double2 *>(p + k + 16 + 2 * u);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s -= c[u].x;
                s -= c[u].y;
            }
            if (k + 48 <= e) {
#pragma unroll
                for (int u = 0; u < 8; ++u) c[u] = *reinterpret_cast<const double2 *>(p + k + 32 + 2 * u);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s -= d[u].x;
                s -= d[u].y;
            }
        }
        if (k + 16 <= e) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s -= c[u].x;
                s -= c[u].y;
            }
            k += 16;
        }
    }
    for (; k < e; ++k) s -= p[k];
    return s;
}
// chain16 with the schedule pinned: the 8 pair reads, then the 16 subtractions, then the copies
__device__ double chain16_sb(double s, const double *p, int a, int e)
{
    int k = a;
    if ((k & 1) && k < e) s -= p[k++];
    if (e - k >= 32) {
        double2 c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = *reinterpret_cast<const double2 *>(p + k + 2 * u);
        for (k += 16; k + 16 <= e; k += 16) {
            double2 n[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) n[u] = *reinterpret_cast<const double2 *>(p + k + 2 * u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s -= c[u].x;
                s -= c[u].y;
            }
            __builtin_amdgcn_sched_barrier(0);
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
// two register sets in turn, schedule pinned (no copies)
__device__ double chain_pp_sb(double s, const double *p, int a, int e)
{
    int k = a;
    if ((k & 1) && k < e) s -= p[k++];
    if (e - k >= 32) {
        double2 c[8], d[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = *reinterpret_cast<const double2 *>(p + k + 2 * u);
        for (; k + 32 <= e; k += 32) {
#pragma unroll
            for (int u = 0; u < 8; ++u) d[u] = *reinterpret_cast<const double2 *>(p + k + 16 + 2 * u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s -= c[u].x;
                s -= c[u].y;
            }
            __builtin_amdgcn_sched_barrier(0);
            // (reads past e stay inside the caller's LDS array: values unused)
#pragma unroll
            for (int u = 0; u < 8; ++u) c[u] = *reinterpret_cast<const double2 *>(p + k + 32 + 2 * u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s -= d[u].x;
                s -= d[u].y;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (k + 16 <= e) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s -= c[u].x;
                s -= c[u].y;
            }
            k += 16;
        }
    }
    for (; k < e; ++k) s -= p[k];
    return s;
}
// 16 in-order subtractions in one asm block: the compiler waits for all 16 operands first, and
// cannot move the next group's reads below them
__device__ __forceinline__ double sub16(double s, const double2 (&c)[8])
{
    asm volatile(
        "v_add_f64 %0, %0, -%1\n\tv_add_f64 %0, %0, -%2\n\tv_add_f64 %0, %0, -%3\n\tv_add_f64 %0, %0, -%4\n\t"
        "v_add_f64 %0, %0, -%5\n\tv_add_f64 %0, %0, -%6\n\tv_add_f64 %0, %0, -%7\n\tv_add_f64 %0, %0, -%8\n\t"
        "v_add_f64 %0, %0, -%9\n\tv_add_f64 %0, %0, -%10\n\tv_add_f64 %0, %0, -%11\n\tv_add_f64 %0, %0, -%12\n\t"
        "v_add_f64 %0, %0, -%13\n\tv_add_f64 %0, %0, -%14\n\tv_add_f64 %0, %0, -%15\n\tv_add_f64 %0, %0, -%16"
        : "+v"(s)
        : "v"(c[0].x), "v"(c[0].y), "v"(c[1].x), "v"(c[1].y), "v"(c[2].x), "v"(c[2].y), "v"(c[3].x), "v"(c[3].y),
          "v"(c[4].x), "v"(c[4].y), "v"(c[5].x), "v"(c[5].y), "v"(c[6].x), "v"(c[6].y), "v"(c[7].x), "v"(c[7].y));
    return s;
}
__device__ double chain_asm(double s, const double *p, int a, int e)
{
    int k = a;
    if ((k & 1) && k < e) s -= p[k++];
    if (e - k >= 32) {
        double2 A[8], B[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) A[u] = *reinterpret_cast<const double2 *>(p + k + 2 * u);
        for (; k + 32 <= e; k += 32) {
#pragma unroll
            for (int u = 0; u < 8; ++u) B[u] = *reinterpret_cast<const double2 *>(p + k + 16 + 2 * u);
            s = sub16(s, A);
            // (the last pass reads up to 16 entries past e: LDS, values unused)
#pragma unroll
            for (int u = 0; u < 8; ++u) A[u] = *reinterpret_cast<const double2 *>(p + k + 32 + 2 * u);
            s = sub16(s, B);
        }
        if (k + 16 <= e) {
            s = sub16(s, A);
            k += 16;
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

// every wave of the block chains its own copy (lane 0): waves sharing a SIMD share its issue
template <int V>
__global__ __launch_bounds__(1024) void kchain(const double *src, double *out, long long *cyc, int m)
{
    __shared__ __attribute__((aligned(16))) double p[M * 4 + 64];
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int t = threadIdx.x; t < M * 4; t += blockDim.x) p[t] = src[t % M];
    __syncthreads();
    double *q = p + (w % 4) * M;
    double s = 1.0;
    long long t0 = 0, t1 = 0;
    if ((threadIdx.x & 63) == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        if (V == 0) s = chain8(s, q, 0, m);
        else if (V == 1) s = chain16(s, q, 0, m);
        else if (V == 3) s = chain_pp(s, q, 0, m);
        else if (V == 4) s = chain16_sb(s, q, 0, m);
        else if (V == 5) s = chain_pp_sb(s, q, 0, m);
        else if (V == 6) s = chain_asm(s, q, 0, m);
        else s = chain_reg(s, q, 0, m);
        out[w] = s;
        t1 = __builtin_amdgcn_s_memtime();
        cyc[w] = t1 - t0;
    }
    (void)nw;
}

int main()
{
    double h[M];
    for (int i = 0; i < M; ++i) h[i] = 1e-3 * ((i * 7919) % 1013) - 0.5;
    double *src, *out;
    long long *cyc;
    CK(hipMalloc(&src, sizeof h));
    CK(hipMalloc(&out, 8 * 16));
    CK(hipMalloc(&cyc, 8 * 16));
    CK(hipMemcpy(src, h, sizeof h, hipMemcpyHostToDevice));
    const char *names[7] = {"8 ahead (engine)", "16 ahead, 16-B reads", "registers (floor)", "16 ahead, two sets",
                            "16 ahead, pinned", "two sets, pinned", "two sets, asm adds"};
    double ref = 0;
    for (int waves : {1, 4, 16})
        for (int v : {0, 1, 6, 2}) {
            long long best = 1LL << 60;
            double s[16];
            for (int rep = 0; rep < 5; ++rep) {
                const dim3 g(1), b(64 * waves);
                if (v == 0) hipLaunchKernelGGL(kchain<0>, g, b, 0, 0, src, out, cyc, M);
                if (v == 1) hipLaunchKernelGGL(kchain<1>, g, b, 0, 0, src, out, cyc, M);
                if (v == 2) hipLaunchKernelGGL(kchain<2>, g, b, 0, 0, src, out, cyc, M);
                if (v == 3) hipLaunchKernelGGL(kchain<3>, g, b, 0, 0, src, out, cyc, M);
                if (v == 4) hipLaunchKernelGGL(kchain<4>, g, b, 0, 0, src, out, cyc, M);
                if (v == 5) hipLaunchKernelGGL(kchain<5>, g, b, 0, 0, src, out, cyc, M);
                if (v == 6) hipLaunchKernelGGL(kchain<6>, g, b, 0, 0, src, out, cyc, M);
                CK(hipDeviceSynchronize());
                long long c[16];
                CK(hipMemcpy(c, cyc, 8 * waves, hipMemcpyDeviceToHost));
                CK(hipMemcpy(s, out, 8 * waves, hipMemcpyDeviceToHost));
                long long mx = 0;
                for (int w = 0; w < waves; ++w) mx = c[w] > mx ? c[w] : mx;
                if (mx < best) best = mx;
            }
            if (v == 0 && waves == 1) ref = s[0];
            bool same = true;
            for (int w = 0; w < waves; ++w) same = same && !memcmp(&s[w], &ref, 8);
            printf("%2d waves  %-24s %8lld s_memtime ticks for %d entries (%.2f per entry)%s\n", waves, names[v], best, M,
                   (double)best / M, v != 2 ? (same ? "  bitwise ok" : "  MISMATCH") : "");
        }
    return 0;
}
