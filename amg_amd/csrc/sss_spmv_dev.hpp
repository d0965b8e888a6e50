// sss_spmv_dev.hpp — device building blocks shared by the SpMV-shaped kernels.
//
// csr_block_rows(): one workgroup = one CSR-adaptive row block (see sss_spmv.hip).  Each
// row's sum is formed from 0.0 in stored CSR order (the reference's order, SSS_utils.c:174 and
// Solve/SSS_cuda.cu:89-92), then handed to `epi(row, sum)`, which writes the result and
// returns this thread's contribution to an optional block reduction.
#pragma once

#include "sss_engine.hpp"

namespace sss {

struct SpmvSmem {
    double v[kTileEntries];
    int c[kTileEntries];
    double red[kBlock / 64];
};

// Fixed-order block reduction (xor butterfly inside the wave, then waves in order).
// Result valid in thread 0.  Must be reached by every thread of the block.
__device__ __forceinline__ double block_sum(double v, double *red)
{
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    return t;
}

__device__ __forceinline__ double block_max(double v, double *red)
{
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t = fmax(t, red[w]);
    return t;
}

// Returns this thread's summed epilogue contribution (0 for idle threads).
template <class Epi>
__device__ __forceinline__ double csr_block_rows(const int *__restrict__ blk, const int *__restrict__ rp,
                                                 const int *__restrict__ ci, const double *__restrict__ v,
                                                 const double *__restrict__ x, SpmvSmem &sm, Epi epi)
{
    const int r0 = blk[blockIdx.x], r1 = blk[blockIdx.x + 1];
    const int k0 = rp[r0], k1 = rp[r1];
    const int cnt = k1 - k0;
    double contrib = 0.0;
    if (cnt <= kTileEntries) {
        for (int k = threadIdx.x; k < cnt; k += kBlock) {
            sm.v[k] = v[k0 + k];
            sm.c[k] = ci[k0 + k];
        }
        __syncthreads();
        const int r = r0 + (int)threadIdx.x;
        if (r < r1) {
            const int a = rp[r] - k0, e = rp[r + 1] - k0;
            double s = 0.0;
            for (int k = a; k < e; ++k) s += sm.v[k] * x[sm.c[k]];
            contrib = epi(r, s);
        }
    } else {
        double s = 0.0;
        for (int base = k0; base < k1; base += kTileEntries) {
            const int m = min(kTileEntries, k1 - base);
            for (int k = threadIdx.x; k < m; k += kBlock) sm.v[k] = v[base + k] * x[ci[base + k]];
            __syncthreads();
            if (threadIdx.x == 0) {
                int k = 0;
                for (; k + 4 <= m; k += 4) {
                    const double p0 = sm.v[k], p1 = sm.v[k + 1], p2 = sm.v[k + 2], p3 = sm.v[k + 3];
                    s += p0;
                    s += p1;
                    s += p2;
                    s += p3;
                }
                for (; k < m; ++k) s += sm.v[k];
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) contrib = epi(r0, s);
    }
    return contrib;
}

}  // namespace sss
