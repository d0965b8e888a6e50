// sss_coarse_direct.hip — direct coarsest-grid solver (engine's throughput coarse mode).
//
// Replaces the coarse CG(beta==1)+GMRES(30) of SSS_amg_coarest_solve (Solve/SSS_cycle.cu:
// 819-846), whose ~1,000 SpMVs per V-cycle dominate the reference's time,
// by an explicit inverse built once per hierarchy and applied as one fp64 GEMV per cycle.
// on Poisson an exact coarse solve reproduces the reference's printed
// residual history.
//
// Build: in-place Gauss-Jordan with partial pivoting on the GPU (one pivot kernel + one
// rank-1 elimination kernel per column, column unscramble at the end).  Apply: one wave per
// row of the inverse, coalesced 8-B loads along the row, shuffle reduction — HBM/MALL-bound
// (n^2 * 8 B per cycle: 203 MB at n = 5,041).
#include "sss_engine.hpp"

#include <vector>

namespace sss {

__global__ __launch_bounds__(1024) void gj_pivot(double *M, int n, int k, double *colbuf, int *swaps)
{
    __shared__ double s_best[1024 / 64];
    __shared__ int s_idx[1024 / 64];
    __shared__ int s_p;
    double best = -1.0;
    int idx = n;
    for (int i = k + threadIdx.x; i < n; i += 1024) {
        const double a = fabs(M[(size_t)i * n + k]);
        if (a > best || (a == best && i < idx)) { best = a; idx = i; }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const double ob = __shfl_xor(best, off, 64);
        const int oi = __shfl_xor(idx, off, 64);
        if (ob > best || (ob == best && oi < idx)) { best = ob; idx = oi; }
    }
    if ((threadIdx.x & 63) == 0) { s_best[threadIdx.x >> 6] = best; s_idx[threadIdx.x >> 6] = idx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = s_best[0];
        int p = s_idx[0];
        for (int w = 1; w < 1024 / 64; ++w)
            if (s_best[w] > b || (s_best[w] == b && s_idx[w] < p)) { b = s_best[w]; p = s_idx[w]; }
        if (p >= n) p = k;
        s_p = p;
        swaps[k] = p;
    }
    __syncthreads();
    const int p = s_p;
    if (p != k)
        for (int j = threadIdx.x; j < n; j += 1024) {
            const double t = M[(size_t)k * n + j];
            M[(size_t)k * n + j] = M[(size_t)p * n + j];
            M[(size_t)p * n + j] = t;
        }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += 1024) colbuf[i] = M[(size_t)i * n + k];
    __syncthreads();
    const double inv = 1.0 / colbuf[k];
    for (int j = threadIdx.x; j < n; j += 1024) M[(size_t)k * n + j] = (j == k) ? inv : M[(size_t)k * n + j] * inv;
}

__global__ __launch_bounds__(256) void gj_eliminate(double *M, int n, int k, const double *__restrict__ colbuf)
{
    const int j = blockIdx.x * 256 + threadIdx.x;
    const int i = blockIdx.y;
    if (j >= n || i == k) return;
    const double f = colbuf[i];
    if (j == k) M[(size_t)i * n + k] = -f * M[(size_t)k * n + k];
    else M[(size_t)i * n + j] -= f * M[(size_t)k * n + j];
}

__global__ __launch_bounds__(256) void gj_unscramble(double *M, int n, const int *__restrict__ swaps)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double *row = M + (size_t)i * n;
    for (int k = n - 1; k >= 0; --k) {
        const int p = swaps[k];
        if (p != k) {
            const double t = row[k];
            row[k] = row[p];
            row[p] = t;
        }
    }
}

__global__ __launch_bounds__(256) void dense_gemv(const double *__restrict__ M, int n, const double *__restrict__ b,
                                                  double *__restrict__ x)
{
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n) return;
    const double *r = M + (size_t)row * n;
    double s = 0.0;
    for (int j = lane; j < n; j += 64) s += r[j] * b[j];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) x[row] = s;
}

int coarse_direct_build(CoarseDirect &cd, const SSS_MAT &A, hipStream_t s)
{
    const int n = A.num_rows;
    std::vector<double> dense((size_t)n * n, 0.0);
    for (int i = 0; i < n; ++i)
        for (int k = A.row_ptr[i]; k < A.row_ptr[i + 1]; ++k) dense[(size_t)i * n + A.col_idx[k]] += A.val[k];
    cd.n = n;
    cd.inv = dev_alloc<double>((size_t)n * n);
    double *colbuf = dev_alloc<double>((size_t)n);
    int *swaps = dev_alloc<int>((size_t)n);
    if (!cd.inv || !colbuf || !swaps) {
        dev_free(colbuf);
        dev_free(swaps);
        return hip_fail(hipErrorOutOfMemory, "hipMalloc(coarse inverse)", __FILE__, __LINE__);
    }
    SSS_HIP(hipMemcpyAsync(cd.inv, dense.data(), sizeof(double) * dense.size(), hipMemcpyHostToDevice, s));
    const dim3 egrid((n + 255) / 256, n);
    for (int k = 0; k < n; ++k) {
        hipLaunchKernelGGL(gj_pivot, dim3(1), dim3(1024), 0, s, cd.inv, n, k, colbuf, swaps);
        hipLaunchKernelGGL(gj_eliminate, egrid, dim3(256), 0, s, cd.inv, n, k, colbuf);
    }
    hipLaunchKernelGGL(gj_unscramble, dim3((n + 255) / 256), dim3(256), 0, s, cd.inv, n, swaps);
    SSS_HIP(hipGetLastError());
    SSS_HIP(hipStreamSynchronize(s));
    dev_free(colbuf);
    dev_free(swaps);
    return 0;
}

void coarse_direct_free(CoarseDirect &cd)
{
    dev_free(cd.inv);
    cd = CoarseDirect();
}

int coarse_direct_apply(const CoarseDirect &cd, const double *b, double *x, hipStream_t s)
{
    ledger_add(8.0 * cd.n * (double)cd.n + 16.0 * cd.n);
    hipLaunchKernelGGL(dense_gemv, dim3((cd.n + 3) / 4), dim3(256), 0, s, cd.inv, cd.n, b, x);
    SSS_HIP(hipGetLastError());
    return 0;
}

}  // namespace sss
