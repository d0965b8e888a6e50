// sss_blas.hip — device BLAS-1 for the AMG-preconditioned CG, fp64.
//
// dot: fixed-order two-level reduction (per-workgroup lane-strided sums + xor tree + waves in
// order into partials, then launch_final_sum), so results are deterministic run to run.  The
// vector updates are elementwise.  All HBM-bound: 16 B per element for a dot, 24 B for an axpy.
#include "sss_engine.hpp"
#include "sss_spmv_dev.hpp"

namespace sss {

constexpr int kDotBlocks = 1024;   // partial sums per dot (fills the chip, fixed order)

__global__ __launch_bounds__(kBlock) void dot_partials(int n, const double *__restrict__ a, const double *__restrict__ b,
                                                       double *__restrict__ partial)
{
    __shared__ double red[kBlock / 64];
    const int per = (n + gridDim.x - 1) / gridDim.x;
    const int lo = blockIdx.x * per, hi = min(n, lo + per);
    double s = 0.0;
    for (int i = lo + (int)threadIdx.x; i < hi; i += kBlock) s += a[i] * b[i];
    const double t = block_sum(s, red);
    if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

int launch_dot(int n, const double *a, const double *b, double *partial, double *out, hipStream_t s)
{
    hipLaunchKernelGGL(dot_partials, dim3(kDotBlocks), dim3(kBlock), 0, s, n, a, b, partial);
    SSS_HIP(hipGetLastError());
    return launch_final_sum(partial, kDotBlocks, out, false, s);
}

// y = y + alpha * x  (alpha read from device memory: *alpha_num / *alpha_den, sign)
__global__ __launch_bounds__(kBlock) void axpy_dev(int n, const double *__restrict__ num, const double *__restrict__ den,
                                                   double sign, const double *__restrict__ x, double *__restrict__ y)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) y[i] += (sign * (*num / *den)) * x[i];
}

// p = z + beta * p, beta = (num - numold) / den (Polak-Ribiere; numold null: Fletcher-Reeves)
__global__ __launch_bounds__(kBlock) void xpby_dev(int n, const double *__restrict__ num, const double *__restrict__ numold,
                                                   const double *__restrict__ den, const double *__restrict__ z,
                                                   double *__restrict__ p)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) {
        const double beta = (numold ? *num - *numold : *num) / *den;
        p[i] = z[i] + beta * p[i];
    }
}

int launch_axpy_ratio(int n, const double *num, const double *den, double sign, const double *x, double *y,
                      hipStream_t s)
{
    hipLaunchKernelGGL(axpy_dev, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, n, num, den, sign, x, y);
    SSS_HIP(hipGetLastError());
    return 0;
}

int launch_xpby_ratio(int n, const double *num, const double *numold, const double *den, const double *z, double *p,
                      hipStream_t s)
{
    hipLaunchKernelGGL(xpby_dev, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, n, num, numold, den, z, p);
    SSS_HIP(hipGetLastError());
    return 0;
}

}  // namespace sss
