// lab_rows.hip — kernel-variant lab for the in-order row chain on long-row (coarse) levels.
// Every variant computes  y_r = b_r - a_{k0} x_{c0} - a_{k1} x_{c1} - ...  in stored order, so
// all must agree bitwise.  Built as a small shared library driven by tools/lab_rows.py.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -shared -fPIC -o tools/liblab_rows.so tools/lab_rows.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

namespace {
constexpr int kB = 256;

__device__ __forceinline__ double chain_sub(double s, const double *p, int a, int e)
{
    int k = a;
    for (; k + 8 <= e; k += 8) {
        const double p0 = p[k], p1 = p[k + 1], p2 = p[k + 2], p3 = p[k + 3];
        const double p4 = p[k + 4], p5 = p[k + 5], p6 = p[k + 6], p7 = p[k + 7];
        s -= p0; s -= p1; s -= p2; s -= p3; s -= p4; s -= p5; s -= p6; s -= p7;
    }
    for (; k < e; ++k) s -= p[k];
    return s;
}

// tile: <= 256 rows / <= 2048 entries per block, products staged by all threads, one thread per row
__global__ __launch_bounds__(kB) void k_tile(const int *blk, const int *rp, const int *ci, const double *v,
                                             const double *x, const double *b, double *y)
{
    __shared__ double sm[2048];
    const int r0 = blk[blockIdx.x], r1 = blk[blockIdx.x + 1];
    const int k0 = rp[r0], k1 = rp[r1];
    if (k1 - k0 <= 2048) {
        for (int kb = k0 + threadIdx.x; kb < k1; kb += 8 * kB) {
            int j[8];
            double a[8], xv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = kb + u * kB;
                j[u] = k < k1 ? ci[k] : 0;
                a[u] = k < k1 ? v[k] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) xv[u] = x[j[u]];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (kb + u * kB < k1) sm[kb + u * kB - k0] = a[u] * xv[u];
        }
        __syncthreads();
        const int r = r0 + threadIdx.x;
        if (r < r1) y[r] = chain_sub(b[r], sm, rp[r] - k0, rp[r + 1] - k0);
    } else {
        double acc = b[r0];
        for (int base = k0; base < k1; base += 2048) {
            const int m = min(2048, k1 - base);
            for (int k = threadIdx.x; k < m; k += kB) sm[k] = v[base + k] * x[ci[base + k]];
            __syncthreads();
            if (threadIdx.x == 0) acc = chain_sub(acc, sm, 0, m);
            __syncthreads();
        }
        if (threadIdx.x == 0) y[r0] = acc;
    }
}

__device__ __forceinline__ void wsync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// wave per row, strip of S entries per wave (S/64 per lane), lane 0 chains; 4 rows per block
template <int S>
__global__ __launch_bounds__(kB) void k_wave(int n, const int *rp, const int *ci, const double *v, const double *x,
                                             const double *b, double *y)
{
    __shared__ double strips[4][S];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + w;
    if (r >= n) return;
    double *st = strips[w];
    const int k0 = rp[r], k1 = rp[r + 1];
    double acc = b[r];
    for (int base = k0; base < k1; base += S) {
        const int m = min(S, k1 - base);
        constexpr int U = S / 64;
        int j[U];
        double a[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = lane + 64 * u;
            j[u] = q < m ? ci[base + q] : 0;
            a[u] = q < m ? v[base + q] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = x[j[u]];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (lane + 64 * u < m) st[lane + 64 * u] = a[u] * xv[u];
        wsync();
        if (lane == 0) acc = chain_sub(acc, st, 0, m);
        wsync();
    }
    if (lane == 0) y[r] = acc;
}

// wave per row with the next strip's loads issued before the current strip's chain
template <int S>
__global__ __launch_bounds__(kB) void k_wave_db(int n, const int *rp, const int *ci, const double *v, const double *x,
                                                const double *b, double *y)
{
    __shared__ double strips[4][S];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + w;
    if (r >= n) return;
    double *st = strips[w];
    const int k0 = rp[r], k1 = rp[r + 1];
    double acc = b[r];
    constexpr int U = S / 64;
    double p[U];
    auto load = [&](int base) {
        const int m = min(S, k1 - base);
        int j[U];
        double a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = lane + 64 * u;
            j[u] = q < m ? ci[base + q] : 0;
            a[u] = q < m ? v[base + q] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = a[u] * x[j[u]];
    };
    if (k0 < k1) load(k0);
    for (int base = k0; base < k1; base += S) {
        const int m = min(S, k1 - base);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (lane + 64 * u < m) st[lane + 64 * u] = p[u];
        wsync();
        if (base + S < k1) load(base + S);   // in flight during the chain
        if (lane == 0) acc = chain_sub(acc, st, 0, m);
        wsync();
    }
    if (lane == 0) y[r] = acc;
}

// R rows per wave, each row strip-mined in S = 512 / R entries per step; L = 64 / R lanes gather a
// row's strip (8 entries per lane per step), then the row's first lane chains it -- one chain
// instruction advances R rows.
template <int R>
__global__ __launch_bounds__(kB) void k_mrow(int n, const int *rp, const int *ci, const double *v, const double *x,
                                             const double *b, double *y)
{
    constexpr int L = 64 / R, S = 512 / R, U = S / L;
    __shared__ double strips[4][R][S];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ri = lane / L, sub = lane % L;
    const int r = (blockIdx.x * 4 + w) * R + ri;
    int k0 = 0, k1 = 0;
    double acc = 0.0;
    if (r < n) k0 = rp[r], k1 = rp[r + 1], acc = b[r];
    int len = k1 - k0;
    for (int off = 32; off > 0; off >>= 1) len = max(len, __shfl_xor(len, off, 64));
    double *st = strips[w][ri];
    for (int base = 0; base < len; base += S) {
        int j[U];
        double a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = k0 + base + sub + L * u;
            j[u] = k < k1 ? ci[k] : 0;
            a[u] = k < k1 ? v[k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double xv = x[j[u]];
            st[sub + L * u] = a[u] * xv;
        }
        wsync();
        if (sub == 0) acc = chain_sub(acc, st, 0, min(S, k1 - k0 - base));
        wsync();
    }
    if (sub == 0 && r < n) y[r] = acc;
}

struct Dev {
    int n = 0, nnz = 0, nblk = 0;
    int *rp = nullptr, *ci = nullptr, *blk = nullptr;
    double *v = nullptr, *x = nullptr, *b = nullptr, *y = nullptr;
} D;
}  // namespace

extern "C" int lab_load(int n, const int *rp, const int *ci, const double *v)
{
    D.n = n;
    D.nnz = rp[n];
    std::vector<int> blk;
    for (int r = 0; r < n;) {
        blk.push_back(r);
        int e = r + 1;
        if (rp[e] - rp[r] <= 2048)
            while (e < n && e - r < kB && rp[e + 1] - rp[r] <= 2048) ++e;
        r = e;
    }
    blk.push_back(n);
    D.nblk = (int)blk.size() - 1;
    std::vector<double> hx(n), hb(n);
    for (int i = 0; i < n; ++i) hx[i] = 1.0 + 1e-3 * (i % 977), hb[i] = 0.5 + 1e-4 * (i % 131);
    if (hipMalloc(&D.rp, sizeof(int) * (n + 1)) || hipMalloc(&D.ci, sizeof(int) * (D.nnz + 8)) ||
        hipMalloc(&D.v, sizeof(double) * (D.nnz + 8)) || hipMalloc(&D.blk, sizeof(int) * blk.size()) ||
        hipMalloc(&D.x, sizeof(double) * n) || hipMalloc(&D.b, sizeof(double) * n) || hipMalloc(&D.y, sizeof(double) * n))
        return 1;
    hipMemcpy(D.rp, rp, sizeof(int) * (n + 1), hipMemcpyHostToDevice);
    hipMemcpy(D.ci, ci, sizeof(int) * D.nnz, hipMemcpyHostToDevice);
    hipMemcpy(D.v, v, sizeof(double) * D.nnz, hipMemcpyHostToDevice);
    hipMemcpy(D.blk, blk.data(), sizeof(int) * blk.size(), hipMemcpyHostToDevice);
    hipMemcpy(D.x, hx.data(), sizeof(double) * n, hipMemcpyHostToDevice);
    hipMemcpy(D.b, hb.data(), sizeof(double) * n, hipMemcpyHostToDevice);
    return 0;
}

extern "C" void lab_free()
{
    hipFree(D.rp), hipFree(D.ci), hipFree(D.v), hipFree(D.blk), hipFree(D.x), hipFree(D.b), hipFree(D.y);
    D = Dev();
}

static void launch(int variant)
{
    const int nw = (D.n + 3) / 4;
    switch (variant) {
    case 0: hipLaunchKernelGGL(k_tile, dim3(D.nblk), dim3(kB), 0, 0, D.blk, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 1: hipLaunchKernelGGL(k_wave<256>, dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 2: hipLaunchKernelGGL(k_wave<512>, dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 3: hipLaunchKernelGGL(k_wave<1024>, dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 4: hipLaunchKernelGGL(k_wave_db<256>, dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 5: hipLaunchKernelGGL(k_wave_db<512>, dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 6: hipLaunchKernelGGL(k_mrow<4>, dim3((D.n + 15) / 16), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 7: hipLaunchKernelGGL(k_mrow<8>, dim3((D.n + 31) / 32), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 8: hipLaunchKernelGGL(k_mrow<16>, dim3((D.n + 63) / 64), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 9: hipLaunchKernelGGL(k_mrow<32>, dim3((D.n + 127) / 128), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    default: break;
    }
}

// returns avg ms; copies y to host
extern "C" double lab_time(int variant, int reps, double *y_out)
{
    hipMemset(D.y, 0, sizeof(double) * D.n);
    launch(variant);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) launch(variant);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(y_out, D.y, sizeof(double) * D.n, hipMemcpyDeviceToHost);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms / reps;
}
