// row_chain_lab.hip -- one long row's stored-order SpMV by one wave (lab only): the one-launch coarse
// CG's worker row chain (two LDS strips, next strip's loads in flight during the chain), the engine's
// wave_row_chain, and the bare chain over products already in LDS; s_memtime cycles and 100 MHz
// wall-clock per entry.  Row: 2,907 entries (the longest row of the coarsest level of 7-pt 400^3)
// into a 3,449-entry x in LDS.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -Iamg_amd/csrc tools/row_chain_lab.hip -o tools/row_chain_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "sss_engine.hpp"
#include "sss_spmv_dev.hpp"

using namespace sss;

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

constexpr int N = 3449, L = 2907;

__device__ __forceinline__ double add16(double s, const double2 (&c)[8])
{
    asm volatile(
        "v_add_f64 %0, %0, %1\n\tv_add_f64 %0, %0, %2\n\tv_add_f64 %0, %0, %3\n\tv_add_f64 %0, %0, %4\n\t"
        "v_add_f64 %0, %0, %5\n\tv_add_f64 %0, %0, %6\n\tv_add_f64 %0, %0, %7\n\tv_add_f64 %0, %0, %8\n\t"
        "v_add_f64 %0, %0, %9\n\tv_add_f64 %0, %0, %10\n\tv_add_f64 %0, %0, %11\n\tv_add_f64 %0, %0, %12\n\t"
        "v_add_f64 %0, %0, %13\n\tv_add_f64 %0, %0, %14\n\tv_add_f64 %0, %0, %15\n\tv_add_f64 %0, %0, %16"
        : "+v"(s)
        : "v"(c[0].x), "v"(c[0].y), "v"(c[1].x), "v"(c[1].y), "v"(c[2].x), "v"(c[2].y), "v"(c[3].x), "v"(c[3].y),
          "v"(c[4].x), "v"(c[4].y), "v"(c[5].x), "v"(c[5].y), "v"(c[6].x), "v"(c[6].y), "v"(c[7].x), "v"(c[7].y));
    return s;
}
__device__ __forceinline__ double chain_asm(double s, const double *p, int e)
{
    int k = 0;
    if (e >= 32) {
        double2 A[8], B[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) A[u] = *reinterpret_cast<const double2 *>(p + 2 * u);
        for (; k + 32 <= e; k += 32) {
#pragma unroll
            for (int u = 0; u < 8; ++u) B[u] = *reinterpret_cast<const double2 *>(p + k + 16 + 2 * u);
            s = add16(s, A);
#pragma unroll
            for (int u = 0; u < 8; ++u) A[u] = *reinterpret_cast<const double2 *>(p + k + 32 + 2 * u);
            s = add16(s, B);
        }
        if (k + 16 <= e) {
            s = add16(s, A);
            k += 16;
        }
    }
    for (; k < e; ++k) s += p[k];
    return s;
}

__device__ __noinline__ double chain_call(double s, const double *p, int m) { return chain_pipe16<false>(s, p, 0, m); }

template <int CALL>
__device__ __forceinline__ double row_chain2(int k0, int k1, const int *__restrict__ ci, const double *__restrict__ v,
                                             const double *x, double *strip0, double *strip1)
{
    constexpr int U = kWaveStage / 64;
    const int lane = threadIdx.x & 63;
    double acc = 0.0;
    int c[U];
    double a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int q = lane + 64 * u, kc = min(k0 + q, k1 - 1);
        c[u] = ci[kc];
        a[u] = k0 + q < k1 ? v[kc] : 0.0;
    }
    int cur = 0;
    for (int base = k0; base < k1; base += kWaveStage) {
        const int m = min(kWaveStage, k1 - base);
        double *buf = cur ? strip1 : strip0;
        if (CALL == 3) {   // branch-free: past the row, a = 0.0 and the column clamped (slots unused)
            double xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) xv[u] = x[c[u]];
#pragma unroll
            for (int u = 0; u < U; ++u) buf[lane + 64 * u] = a[u] * xv[u];
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = lane + 64 * u;
                if (q < m) buf[q] = a[u] * x[c[u]];
            }
        }
        wave_sync();
        const int nb = base + kWaveStage;
        if (nb < k1) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = lane + 64 * u, kc = min(nb + q, k1 - 1);
                c[u] = ci[kc];
                a[u] = nb + q < k1 ? v[kc] : 0.0;
            }
        }
        if (lane == 0)
            acc = CALL == 1 ? chain_call(acc, buf, m) : CALL >= 2 ? chain_asm(acc, buf, m) : chain_pipe16<false>(acc, buf, 0, m);
        cur ^= 1;
    }
    return acc;
}

// the row's column indices and values reach LDS by LDS-DMA (global_load_lds, no VGPRs), NS strips
// of SW entries ahead; products into one strip, lane 0 chains it
constexpr int SW = 128, NS = 3;
__device__ __forceinline__ void glds_strip(const int *ci, const double *v, int base, int k1, int *cis, unsigned *vs)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < SW / 64; ++j)
        __builtin_amdgcn_global_load_lds(ci + min(base + 64 * j + lane, k1 - 1), cis + 64 * j, 4, 0, 0);
    const unsigned *vu = reinterpret_cast<const unsigned *>(v);
#pragma unroll
    for (int j = 0; j < 2 * SW / 64; ++j)
        __builtin_amdgcn_global_load_lds(vu + min(2 * base + 64 * j + lane, 2 * k1 - 1), vs + 64 * j, 4, 0, 0);
}
constexpr int kGldsPerStrip = SW / 64 + 2 * SW / 64;
__device__ __forceinline__ double row_chain_glds(int k0, int k1, const int *__restrict__ ci, const double *__restrict__ v,
                                                 const double *x, int *cis, unsigned *vs, double *buf)
{
    const int lane = threadIdx.x & 63;
    double acc = 0.0;
    const int ns = (k1 - k0 + SW - 1) / SW;
    for (int i = 0; i < NS - 1 && i < ns; ++i) glds_strip(ci, v, k0 + i * SW, k1, cis + i * SW, vs + 2 * i * SW);
    for (int i = 0; i < ns; ++i) {
        const int st = i % NS, base = k0 + i * SW, m = min(SW, k1 - base);
        // strip i landed: the strips issued after it may stay in flight
        if (i + 1 < ns) __builtin_amdgcn_s_waitcnt(0x0F70 | kGldsPerStrip);   // vmcnt(kGldsPerStrip)
        else __builtin_amdgcn_s_waitcnt(0x0F70);                              // vmcnt(0)
        const int *cs = cis + st * SW;
        const double *vd = reinterpret_cast<const double *>(vs + 2 * st * SW);
#pragma unroll
        for (int u = 0; u < SW / 64; ++u) {
            const int q = lane + 64 * u;
            if (q < m) buf[q] = vd[q] * x[cs[q]];
        }
        wave_sync();
        if (i + NS - 1 < ns)
            glds_strip(ci, v, k0 + (i + NS - 1) * SW, k1, cis + ((i + NS - 1) % NS) * SW, vs + 2 * ((i + NS - 1) % NS) * SW);
        if (lane == 0) acc = chain_pipe16<false>(acc, buf, 0, m);
        wave_sync();
    }
    return acc;
}

template <int V>
__global__ __launch_bounds__(1024) void krow(const int *ci, const double *v, const double *xg, double *out,
                                             long long *cyc)
{
    __shared__ __attribute__((aligned(16))) double x[4096];
    __shared__ __attribute__((aligned(16))) double st[16 * 2 * kWaveStage];
    __shared__ __attribute__((aligned(16))) double pr[L + 40];
    for (int i = threadIdx.x; i < N; i += blockDim.x) x[i] = xg[i];
    if (V == 2)
        for (int i = threadIdx.x; i < L; i += blockDim.x) pr[i] = v[i] * xg[ci[i]];
    __syncthreads();
    if (threadIdx.x >= 64) return;   // one wave works; the rest of the block has left
    const long long t0 = __builtin_amdgcn_s_memtime(), w0 = wall_clock64();
    double s = 0;
    if (V == 0) s = row_chain2<0>(0, L, ci, v, x, st, st + kWaveStage);
    if (V == 3) s = row_chain2<1>(0, L, ci, v, x, st, st + kWaveStage);
    if (V == 5) s = row_chain2<2>(0, L, ci, v, x, st, st + kWaveStage);
    if (V == 6 && threadIdx.x == 0) s = chain_asm(0.0, pr, L);
    if (V == 7) s = row_chain2<3>(0, L, ci, v, x, st, st + kWaveStage);
    if (V == 4) {
        int *cis = reinterpret_cast<int *>(st);
        unsigned *vs = reinterpret_cast<unsigned *>(st + NS * SW);
        s = row_chain_glds(0, L, ci, v, x, cis, vs, st + NS * SW + NS * SW * 2);
    }
    if (V == 1) s = wave_row_chain<false>(0, L, ci, v, [&](int col, double a) { return a * x[col]; }, 0.0, st);
    if (V == 2 && threadIdx.x == 0) s = chain_pipe16<false>(0.0, pr, 0, L);
    if (threadIdx.x == 0) {
        out[0] = s;
        cyc[0] = __builtin_amdgcn_s_memtime() - t0;
        cyc[1] = wall_clock64() - w0;
    }
}

int main()
{
    int *hc = new int[L];
    double *hv = new double[L], *hx = new double[N];
    for (int i = 0; i < L; ++i) hc[i] = (int)((i * 7919LL) % N), hv[i] = 1e-3 * ((i * 31) % 977) - 0.4;
    for (int i = 0; i < N; ++i) hx[i] = 1.0 + 1e-4 * (i % 113);
    int *ci;
    double *v, *xg, *out;
    long long *cyc;
    CK(hipMalloc(&ci, 4 * L));
    CK(hipMalloc(&v, 8 * L));
    CK(hipMalloc(&xg, 8 * N));
    CK(hipMalloc(&out, 8));
    CK(hipMalloc(&cyc, 16));
    CK(hipMemcpy(ci, hc, 4 * L, hipMemcpyHostToDevice));
    CK(hipMemcpy(v, hv, 8 * L, hipMemcpyHostToDevice));
    CK(hipMemcpy(xg, hx, 8 * N, hipMemcpyHostToDevice));
    const char *names[8] = {"worker row chain (2 strips)", "wave_row_chain", "bare chain over LDS",
                            "2 strips, chain not inlined", "LDS-DMA strips (3 x 128)",
                            "2 strips, asm chain", "bare asm chain over LDS",
                            "2 strips, asm chain, flat products"};
    double ref = 0;
    for (int v_ = 0; v_ < 8; ++v_) {
        long long best[2] = {1LL << 60, 1LL << 60};
        double s = 0;
        for (int rep = 0; rep < 7; ++rep) {
            if (v_ == 0) hipLaunchKernelGGL(krow<0>, dim3(1), dim3(1024), 0, 0, ci, v, xg, out, cyc);
            if (v_ == 1) hipLaunchKernelGGL(krow<1>, dim3(1), dim3(1024), 0, 0, ci, v, xg, out, cyc);
            if (v_ == 2) hipLaunchKernelGGL(krow<2>, dim3(1), dim3(1024), 0, 0, ci, v, xg, out, cyc);
            if (v_ == 5) hipLaunchKernelGGL(krow<5>, dim3(1), dim3(1024), 0, 0, ci, v, xg, out, cyc);
            if (v_ == 7) hipLaunchKernelGGL(krow<7>, dim3(1), dim3(1024), 0, 0, ci, v, xg, out, cyc);
            if (v_ == 6) hipLaunchKernelGGL(krow<6>, dim3(1), dim3(1024), 0, 0, ci, v, xg, out, cyc);
            if (v_ == 4) hipLaunchKernelGGL(krow<4>, dim3(1), dim3(1024), 0, 0, ci, v, xg, out, cyc);
            if (v_ == 3) hipLaunchKernelGGL(krow<3>, dim3(1), dim3(1024), 0, 0, ci, v, xg, out, cyc);
            CK(hipDeviceSynchronize());
            long long c[2];
            CK(hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&s, out, 8, hipMemcpyDeviceToHost));
            if (c[0] < best[0]) best[0] = c[0], best[1] = c[1];
        }
        if (v_ == 0) ref = s;
        printf("%-30s %7lld cycles (%.2f per entry), %.2f us (%.2f ns per entry)%s\n", names[v_], best[0],
               (double)best[0] / L, best[1] * 0.01, best[1] * 10.0 / L, memcmp(&s, &ref, 8) ? "  MISMATCH" : "  bitwise ok");
    }
    return 0;
}
