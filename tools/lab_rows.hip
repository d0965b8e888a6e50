// lab_rows.hip — kernel-variant lab for the in-order row chain on long-row (coarse) levels.
// Every variant computes  y_r = b_r - a_{k0} x_{c0} - a_{k1} x_{c1} - ...  in stored order, so
// all must agree bitwise.  Built as a small shared library driven by tools/lab_rows.py.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -shared -fPIC -o tools/liblab_rows.so tools/lab_rows.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
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
// chain with the next 8 LDS reads in flight while the current 8 are subtracted
__device__ __forceinline__ double chain_sub_pipe(double s, const double *p, int a, int e)
{
    int k = a;
    if (e - a >= 16) {
        double c0 = p[k], c1 = p[k + 1], c2 = p[k + 2], c3 = p[k + 3];
        double c4 = p[k + 4], c5 = p[k + 5], c6 = p[k + 6], c7 = p[k + 7];
        for (; k + 16 <= e; k += 8) {
            const double n0 = p[k + 8], n1 = p[k + 9], n2 = p[k + 10], n3 = p[k + 11];
            const double n4 = p[k + 12], n5 = p[k + 13], n6 = p[k + 14], n7 = p[k + 15];
            s -= c0; s -= c1; s -= c2; s -= c3; s -= c4; s -= c5; s -= c6; s -= c7;
            c0 = n0, c1 = n1, c2 = n2, c3 = n3, c4 = n4, c5 = n5, c6 = n6, c7 = n7;
        }
        s -= c0; s -= c1; s -= c2; s -= c3; s -= c4; s -= c5; s -= c6; s -= c7;
        k += 8;
    }
    for (; k < e; ++k) s -= p[k];
    return s;
}

template <bool PIPE>
__device__ __forceinline__ double chain_x(double s, const double *p, int a, int e)
{
    return PIPE ? chain_sub_pipe(s, p, a, e) : chain_sub(s, p, a, e);
}

template <bool PIPE = false>
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
        if (r < r1) y[r] = chain_x<PIPE>(b[r], sm, rp[r] - k0, rp[r + 1] - k0);
    } else {
        double acc = b[r0];
        for (int base = k0; base < k1; base += 2048) {
            const int m = min(2048, k1 - base);
            for (int k = threadIdx.x; k < m; k += kB) sm[k] = v[base + k] * x[ci[base + k]];
            __syncthreads();
            if (threadIdx.x == 0) acc = chain_x<PIPE>(acc, sm, 0, m);
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
template <int S, bool PIPE = false>
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
        if (lane == 0) acc = chain_x<PIPE>(acc, st, 0, m);
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


// lane per row, K entries of every row per chunk: the wave's 4*16 lanes... each of the 64 lanes
// owns one row.  Loads are coalesced across rows (K consecutive entries of a row per K lanes),
// products land in LDS at [row][k] (stride K+1: conflict-free column reads), then every lane
// chains its own row's K products.  PF: the next chunk's products are formed in registers
// before the current chunk is chained.
template <int K, bool PF>
__global__ __launch_bounds__(kB) void k_lanerow(int n, const int *rp, const int *ci, const double *v,
                                                const double *x, const double *b, double *y)
{
    constexpr int U = K;                 // entries per lane per chunk (64 rows * K / 64 lanes)
    constexpr int RPI = 64 / K;          // rows covered by one load instruction
    __shared__ double st[4][64 * (K + 1)];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int rbase = (blockIdx.x * 4 + w) * 64;
    const int r = rbase + lane;
    int k0 = 0, k1 = 0;
    double acc = 0.0;
    if (r < n) k0 = rp[r], k1 = rp[r + 1], acc = b[r];
    const int len = k1 - k0;
    int mx = len;
    for (int off = 32; off > 0; off >>= 1) mx = max(mx, __shfl_xor(mx, off, 64));
    // load mapping: instruction u covers rows u*RPI + lane/K, entry lane%K of the chunk
    const int sub = lane % K;
    int ls[U], ll[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int rr = u * RPI + lane / K;
        ls[u] = __shfl(k0, rr, 64);
        ll[u] = __shfl(len, rr, 64);
    }
    double *sw = st[w];
    double p[U];
    auto load = [&](int c) {
        int j[U];
        double a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = c + sub;
            j[u] = q < ll[u] ? ci[ls[u] + q] : -1;
            a[u] = q < ll[u] ? v[ls[u] + q] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = j[u] >= 0 ? a[u] * x[j[u]] : 0.0;
    };
    if (PF && mx > 0) load(0);
    for (int c = 0; c < mx; c += K) {
        if (!PF) load(c);
#pragma unroll
        for (int u = 0; u < U; ++u) sw[(u * RPI + lane / K) * (K + 1) + sub] = p[u];
        wsync();
        if (PF && c + K < mx) load(c + K);
        const int e = min(K, len - c);
        const double *row = sw + lane * (K + 1);
        for (int k = 0; k < e; ++k) acc -= row[k];
        wsync();
    }
    if (r < n) y[r] = acc;
}

// tile with column-sorted staging: within each staged segment (the block's tile, or a 2048 chunk
// of a long row) entries are stored sorted by column, packed (col << 11) | pos, pos = stored-order
// position in the segment; products land at their stored position, the chain is unchanged
template <bool PIPE = false>
__global__ __launch_bounds__(kB) void k_tile_sorted(const int *blk, const int *rp, const int *pk, const double *v,
                                                    const double *x, const double *b, double *y)
{
    __shared__ double sm[2048];
    const int r0 = blk[blockIdx.x], r1 = blk[blockIdx.x + 1];
    const int k0 = rp[r0], k1 = rp[r1];
    if (k1 - k0 <= 2048) {
        const int r = r0 + threadIdx.x;
        int ra = 0, re = 0;
        double br = 0.0;
        if (r < r1) ra = rp[r], re = rp[r + 1], br = b[r];
        for (int kb = k0 + threadIdx.x; kb < k1; kb += 8 * kB) {
            int j[8];
            double a[8], xv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = kb + u * kB;
                j[u] = k < k1 ? pk[k] : 0;
                a[u] = k < k1 ? v[k] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) xv[u] = x[j[u] >> 11];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (kb + u * kB < k1) sm[j[u] & 2047] = a[u] * xv[u];
        }
        __syncthreads();
        if (r < r1) y[r] = chain_x<PIPE>(br, sm, ra - k0, re - k0);
    } else {
        double acc = b[r0];
        for (int base = k0; base < k1; base += 2048) {
            const int m = min(2048, k1 - base);
            for (int k = threadIdx.x; k < m; k += kB) {
                const int q = pk[base + k];
                sm[q & 2047] = v[base + k] * x[q >> 11];
            }
            __syncthreads();
            if (threadIdx.x == 0) acc = chain_x<PIPE>(acc, sm, 0, m);
            __syncthreads();
        }
        if (threadIdx.x == 0) y[r0] = acc;
    }
}

// wave per row (as k_wave_db<256>) with each 256-entry strip column-sorted, packed (col << 8) | pos
__global__ __launch_bounds__(kB) void k_wave_sorted(int n, const int *rp, const int *pk, const double *v,
                                                    const double *x, const double *b, double *y)
{
    constexpr int S = 256, U = 4;
    __shared__ double strips[4][S];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + w;
    if (r >= n) return;
    double *st = strips[w];
    const int k0 = rp[r], k1 = rp[r + 1];
    double acc = b[r];
    double p[U];
    int pos[U];
    auto load = [&](int base) {
        const int m = min(S, k1 - base);
        int j[U];
        double a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = lane + 64 * u;
            j[u] = q < m ? pk[base + q] : -1;
            a[u] = q < m ? v[base + q] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            p[u] = j[u] >= 0 ? a[u] * x[j[u] >> 8] : 0.0;
            pos[u] = j[u] >= 0 ? (j[u] & 255) : -1;
        }
    };
    if (k0 < k1) load(k0);
    for (int base = k0; base < k1; base += S) {
        const int m = min(S, k1 - base);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (pos[u] >= 0) st[pos[u]] = p[u];
        wsync();
        if (base + S < k1) load(base + S);
        if (lane == 0) acc = chain_sub(acc, st, 0, m);
        wsync();
    }
    if (lane == 0) y[r] = acc;
}

// generalised sorted tile: T entries per tile, NT threads, rows per block <= NT, packed
// (col << log2 T) | pos; NOLOAD: products are synthetic (chain cost alone)
template <int T, int NT, bool NOLOAD = false>
__global__ __launch_bounds__(NT) void k_tsort(const int *blk, const int *rp, const unsigned *pk, const double *v,
                                              const double *x, const double *b, double *y)
{
    constexpr int SH = __builtin_ctz(T);
    constexpr unsigned MASK = T - 1;
    __shared__ double sm[T];
    const int r0 = blk[blockIdx.x], r1 = blk[blockIdx.x + 1];
    const int k0 = rp[r0], k1 = rp[r1];
    if (k1 - k0 <= T) {
        const int r = r0 + threadIdx.x;
        int ra = 0, re = 0;
        double br = 0.0;
        if (r < r1) ra = rp[r], re = rp[r + 1], br = b[r];
        if (NOLOAD) {
            for (int k = threadIdx.x; k < k1 - k0; k += NT) sm[k] = 1e-3 * k;
        } else {
            for (int kb = k0 + threadIdx.x; kb < k1; kb += 8 * NT) {
                unsigned j[8];
                double a[8], xv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int k = kb + u * NT;
                    j[u] = k < k1 ? pk[k] : 0u;
                    a[u] = k < k1 ? v[k] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) xv[u] = x[j[u] >> SH];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (kb + u * NT < k1) sm[j[u] & MASK] = a[u] * xv[u];
            }
        }
        __syncthreads();
        if (r < r1) y[r] = chain_sub(br, sm, ra - k0, re - k0);
    } else {
        double acc = b[r0];
        for (int base = k0; base < k1; base += T) {
            const int m = min(T, k1 - base);
            for (int k = threadIdx.x; k < m; k += NT) {
                const unsigned q = pk[base + k];
                sm[q & MASK] = NOLOAD ? 1e-3 * k : v[base + k] * x[q >> SH];
            }
            __syncthreads();
            if (threadIdx.x == 0) acc = chain_sub(acc, sm, 0, m);
            __syncthreads();
        }
        if (threadIdx.x == 0) y[r0] = acc;
    }
}

struct SortedCfg {
    int T = 0, NT = 0, nblk = 0;
    int *blk = nullptr;
    unsigned *pk = nullptr;
    double *v = nullptr;
};

// CSR-vector (throughput mode: NOT the reference's summation order): G lanes per row, lane g
// accumulates entries g, g+G, ... (U loads in flight), xor-shuffle reduction inside the group.
template <int G, int U>
__global__ __launch_bounds__(kB) void k_vec(int n, const int *rp, const int *ci, const double *v, const double *x,
                                            const double *b, double *y)
{
    const int r = blockIdx.x * (kB / G) + (int)threadIdx.x / G, g = threadIdx.x % G;
    int k0 = 0, k1 = 0;
    if (r < n) k0 = rp[r], k1 = rp[r + 1];
    double s0 = 0.0, s1 = 0.0;
    for (int k = k0 + g; k < k1; k += G * U) {
        int j[U];
        double a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int kk = k + u * G;
            j[u] = kk < k1 ? ci[kk] : -1;
            a[u] = kk < k1 ? v[kk] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double xv = j[u] >= 0 ? x[j[u]] : 0.0;
            if (u & 1) s1 += a[u] * xv; else s0 += a[u] * xv;
        }
    }
    double s = s0 + s1;
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (r < n && g == 0) y[r] = b[r] - s;
}

// x staged in LDS, column-chunked (throughput mode: free order).  Columns are cut into chunks of K;
// the matrix is stored chunk-major (for chunk c a CSR over all rows with 16-bit chunk-local
// columns, rows column-sorted).  A persistent workgroup owns the rows [rs[b], rs[b+1]) (balanced
// by nnz); for every chunk it stages x[cK, cK + K) in LDS, then each wave takes R consecutive rows
// at a time, lane-strided over the row's chunk entries with R*Q loads in flight, one xor-reduction
// per row and chunk, the running row sum kept in LDS by the owning wave.
constexpr int kLxRows = 2048;   // max rows per workgroup
template <int K, int NT, int R, int Q>
__global__ __launch_bounds__(NT) void k_ldsx(int n, int nchunk, const int *rs, const int *crp,
                                             const unsigned short *cci, const double *cv, const double *x,
                                             const double *b, double *y)
{
    __shared__ double xs[K];
    __shared__ double acc[kLxRows];
    constexpr int NW = NT / 64;
    const int r0 = rs[blockIdx.x], r1 = rs[blockIdx.x + 1];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int c = 0; c < nchunk; ++c) {
        const int cbase = c * K, cn = min(K, n - cbase);
        __syncthreads();
        for (int i = threadIdx.x; i < cn; i += NT) xs[i] = x[cbase + i];
        __syncthreads();
        const int *rp = crp + (size_t)c * (n + 1);
        for (int rb = r0 + wave * R; rb < r1; rb += NW * R) {
            int k0[R], k1[R];
            double s[R];
            int len = 0;
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int r = rb + u;
                k0[u] = r < r1 ? rp[r] : 0;
                k1[u] = r < r1 ? rp[r + 1] : 0;
                len = max(len, k1[u] - k0[u]);
                s[u] = 0.0;
            }
            for (int t = lane; t < len; t += 64 * Q) {
                unsigned short cc[R][Q];
                double aa[R][Q];
#pragma unroll
                for (int u = 0; u < R; ++u)
#pragma unroll
                    for (int q = 0; q < Q; ++q) {
                        const int k = k0[u] + t + 64 * q;
                        const bool ok = k < k1[u];
                        cc[u][q] = ok ? cci[k] : (unsigned short)0;
                        aa[u][q] = ok ? cv[k] : 0.0;
                    }
#pragma unroll
                for (int u = 0; u < R; ++u)
#pragma unroll
                    for (int q = 0; q < Q; ++q) s[u] += aa[u][q] * xs[cc[u][q]];
            }
#pragma unroll
            for (int u = 0; u < R; ++u) {
                double v = s[u];
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
                const int r = rb + u;
                if (lane == 0 && r < r1) {
                    const double tot = c == 0 ? v : acc[r - r0] + v;
                    if (c + 1 == nchunk) y[r] = b[r] - tot;
                    else acc[r - r0] = tot;
                }
            }
        }
    }
}

// Merged row groups (throughput mode: free order): G consecutive rows' entries merged into one
// column-sorted list, packed (col << 5) | row-in-group.  One wave per group, lane-strided over the
// list with U loads in flight; per-lane accumulator per row (select chain), xor-reduced per row.
// Neighbouring rows share most columns, so 64 consecutive merged entries touch ~G x fewer lines.
template <int G, int U>
__global__ __launch_bounds__(kB) void k_merged(int n, const int *gp, const unsigned *mk, const double *mv,
                                               const double *x, const double *b, double *y)
{
    const int g = blockIdx.x * (kB / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int ng = (n + G - 1) / G;
    if (g >= ng) return;
    const int k0 = gp[g], k1 = gp[g + 1];
    double s[G];
#pragma unroll
    for (int u = 0; u < G; ++u) s[u] = 0.0;
    for (int k = k0 + lane; k < k1; k += 64 * U) {
        unsigned q[U];
        double a[U];
#pragma unroll
        for (int t = 0; t < U; ++t) {
            const int kk = k + 64 * t;
            q[t] = kk < k1 ? mk[kk] : 0u;
            a[t] = kk < k1 ? mv[kk] : 0.0;
        }
#pragma unroll
        for (int t = 0; t < U; ++t) {
            const double p = a[t] * x[q[t] >> 5];
            const unsigned rid = q[t] & 31u;
#pragma unroll
            for (int u = 0; u < G; ++u) s[u] += rid == (unsigned)u ? p : 0.0;
        }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
        double v = s[u];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        const int r = g * G + u;
        if (lane == 0 && r < n) y[r] = b[r] - v;
    }
}

// Merged groups with LDS accumulators: one workgroup per group of G rows, its 4 waves take quarters
// of the merged list; each lane accumulates into its private LDS slot acc[w][row][lane] (no select
// chain, so G can grow: fewer x lines per 64 gathers), then per-row lane trees and waves in order.
template <int G>
__global__ __launch_bounds__(kB) void k_mlds(int n, const int *gp, const unsigned *mk, const double *mv,
                                             const double *x, const double *b, double *y)
{
    __shared__ double acc[4][G][64];
    __shared__ double red[4][G];
    const int g = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int k0 = gp[g], k1 = gp[g + 1], len = k1 - k0, per = (len + 3) >> 2;
    const int a = k0 + min(len, w * per), e = k0 + min(len, (w + 1) * per);
#pragma unroll
    for (int u = 0; u < G; ++u) acc[w][u][lane] = 0.0;
    constexpr int U = 4;
    for (int k = a + lane; k < e; k += 64 * U) {
        unsigned q[U];
        double av[U];
#pragma unroll
        for (int t = 0; t < U; ++t) {
            const int kk = k + 64 * t;
            q[t] = kk < e ? mk[kk] : 0u;
            av[t] = kk < e ? mv[kk] : 0.0;
        }
#pragma unroll
        for (int t = 0; t < U; ++t) {
            if (k + 64 * t >= e) break;
            const double p = av[t] * x[q[t] >> 5];
            acc[w][q[t] & 31u][lane] += p;
        }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
        double v = acc[w][u][lane];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0) red[w][u] = v;
    }
    __syncthreads();
    if (threadIdx.x < G) {
        const int u = threadIdx.x, r = g * G + u;
        const double t = ((red[0][u] + red[1][u]) + red[2][u]) + red[3][u];
        if (r < n) y[r] = b[r] - t;
    }
}

struct Lx {
    int K = 0, nchunk = 0, nb = 0;
    int *rs = nullptr, *crp = nullptr;
    unsigned short *cci = nullptr;
    double *cv = nullptr;
};

struct Merged {
    int G = 0;
    int *gp = nullptr;
    unsigned *mk = nullptr;
    double *mv = nullptr;
};

struct Dev {
    int n = 0, nnz = 0, nblk = 0;
    Lx lx[2];   // K = 8192, 16384
    Merged mg[5];   // G = 4, 8, 16, 32, 16(b)
    int *rp = nullptr, *ci = nullptr, *blk = nullptr, *pk11 = nullptr, *pk8 = nullptr;
    double *v11 = nullptr, *v8 = nullptr;
    std::vector<int> hrp, hci;
    std::vector<double> hv;
    SortedCfg cfg[4];   // T = 2048, 4096, 8192, 16384
    int *rci = nullptr;        // row-sorted copies
    double *rv = nullptr;
    double *v = nullptr, *x = nullptr, *b = nullptr, *y = nullptr;
} D;
}  // namespace

extern "C" int lab_load(int n, const int *rp, const int *ci, const double *v)
{
    D.n = n;
    D.nnz = rp[n];
    D.hrp.assign(rp, rp + n + 1), D.hci.assign(ci, ci + D.nnz), D.hv.assign(v, v + D.nnz);
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
    // column-sorted segments (tile: 2048-entry segments of blocks; wave: 256-entry strips of rows)
    auto sorted = [&](int shift, auto segs, std::vector<int> &pk, std::vector<double> &vs) {
        pk.assign(D.nnz, 0), vs.assign(D.nnz, 0.0);
        std::vector<int> idx;
        segs([&](int a, int e) {
            idx.resize(e - a);
            for (int t = 0; t < e - a; ++t) idx[t] = a + t;
            std::stable_sort(idx.begin(), idx.end(), [&](int p, int q) { return ci[p] < ci[q]; });
            for (int t = 0; t < e - a; ++t) pk[a + t] = (ci[idx[t]] << shift) | (idx[t] - a), vs[a + t] = v[idx[t]];
        });
    };
    std::vector<int> pk11, pk8;
    std::vector<double> v11, v8;
    const bool ok11 = n < (1 << 20), ok8 = n < (1 << 23);
    if (ok11)
        sorted(11, [&](auto f) {
            for (int bI = 0; bI < D.nblk; ++bI) {
                const int a = rp[blk[bI]], e = rp[blk[bI + 1]];
                for (int s = a; s < e; s += 2048) f(s, std::min(e, s + 2048));
            }
        }, pk11, v11);
    if (ok8)
        sorted(8, [&](auto f) {
            for (int r = 0; r < n; ++r)
                for (int s = rp[r]; s < rp[r + 1]; s += 256) f(s, std::min(rp[r + 1], s + 256));
        }, pk8, v8);
    auto up = [](auto *&d, const auto &h) {
        if (h.empty()) return;
        hipMalloc(&d, sizeof(h[0]) * h.size());
        hipMemcpy(d, h.data(), sizeof(h[0]) * h.size(), hipMemcpyHostToDevice);
    };
    up(D.pk11, pk11), up(D.v11, v11), up(D.pk8, pk8), up(D.v8, v8);
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
    for (auto &c : D.cfg) hipFree(c.blk), hipFree(c.pk), hipFree(c.v);
    for (auto &L : D.lx) hipFree(L.rs), hipFree(L.crp), hipFree(L.cci), hipFree(L.cv);
    for (auto &M : D.mg) hipFree(M.gp), hipFree(M.mk), hipFree(M.mv);
    hipFree(D.rci), hipFree(D.rv);
    hipFree(D.pk11), hipFree(D.pk8), hipFree(D.v11), hipFree(D.v8);
    hipFree(D.rp), hipFree(D.ci), hipFree(D.v), hipFree(D.blk), hipFree(D.x), hipFree(D.b), hipFree(D.y);
    D = Dev();
}

static void row_sorted()
{
    if (D.rci) return;
    std::vector<int> c(D.nnz), idx;
    std::vector<double> w(D.nnz);
    for (int r = 0; r < D.n; ++r) {
        const int a = D.hrp[r], e = D.hrp[r + 1];
        idx.resize(e - a);
        for (int t = 0; t < e - a; ++t) idx[t] = a + t;
        std::stable_sort(idx.begin(), idx.end(), [&](int p, int q) { return D.hci[p] < D.hci[q]; });
        for (int t = 0; t < e - a; ++t) c[a + t] = D.hci[idx[t]], w[a + t] = D.hv[idx[t]];
    }
    hipMalloc(&D.rci, sizeof(int) * (D.nnz + 8));
    hipMalloc(&D.rv, sizeof(double) * (D.nnz + 8));
    hipMemcpy(D.rci, c.data(), sizeof(int) * D.nnz, hipMemcpyHostToDevice);
    hipMemcpy(D.rv, w.data(), sizeof(double) * D.nnz, hipMemcpyHostToDevice);
}

// chunk-major copy for k_ldsx: rows column-sorted, cut at multiples of K; nb row ranges of ~equal nnz
static Lx *lx_get(int slot, int K, int nb)
{
    Lx &L = D.lx[slot];
    if (L.K) return &L;
    const int n = D.n;
    if (n > 16 * 65536) return nullptr;
    nb = std::max(nb, (n + kLxRows - 1) / kLxRows);
    const int nc = (n + K - 1) / K;
    std::vector<int> crp((size_t)nc * (n + 1), 0), cnt((size_t)nc * n, 0);
    const int *rp = D.hrp.data(), *ci = D.hci.data();
    for (int r = 0; r < n; ++r)
        for (int k = rp[r]; k < rp[r + 1]; ++k) cnt[(size_t)(ci[k] / K) * n + r]++;
    std::vector<long long> base(nc + 1, 0);
    for (int c = 0; c < nc; ++c) {
        long long s = 0;
        for (int r = 0; r < n; ++r) s += cnt[(size_t)c * n + r];
        base[c + 1] = base[c] + s;
    }
    // crp holds absolute positions into the concatenated chunk arrays
    for (int c = 0; c < nc; ++c) {
        long long p = base[c];
        for (int r = 0; r < n; ++r) {
            crp[(size_t)c * (n + 1) + r] = (int)p;
            p += cnt[(size_t)c * n + r];
        }
        crp[(size_t)c * (n + 1) + n] = (int)p;
    }
    std::vector<unsigned short> cc(D.nnz);
    std::vector<double> vv(D.nnz);
    std::vector<int> fill(crp);
    std::vector<int> idx;
    for (int r = 0; r < n; ++r) {
        idx.resize(rp[r + 1] - rp[r]);
        for (int t = 0; t < (int)idx.size(); ++t) idx[t] = rp[r] + t;
        std::stable_sort(idx.begin(), idx.end(), [&](int p, int q) { return ci[p] < ci[q]; });
        for (int k : idx) {
            const int c = ci[k] / K;
            const int pos = fill[(size_t)c * (n + 1) + r]++;
            cc[pos] = (unsigned short)(ci[k] - c * K);
            vv[pos] = D.hv[k];
        }
    }
    std::vector<int> rs(1, 0);
    const double per = (double)D.nnz / nb;
    for (int r = 0, b = 1; r < n && b < nb; ++r)
        if ((double)rp[r + 1] >= per * b || r + 1 - rs.back() >= kLxRows) rs.push_back(r + 1), ++b;
    while (rs.back() < n) {   // cap the last ranges at kLxRows rows
        const int nx = std::min(n, rs.back() + kLxRows);
        rs.push_back(nx);
    }
    L.K = K, L.nchunk = nc, L.nb = (int)rs.size() - 1;
    hipMalloc(&L.rs, sizeof(int) * rs.size());
    hipMemcpy(L.rs, rs.data(), sizeof(int) * rs.size(), hipMemcpyHostToDevice);
    hipMalloc(&L.crp, sizeof(int) * crp.size());
    hipMemcpy(L.crp, crp.data(), sizeof(int) * crp.size(), hipMemcpyHostToDevice);
    hipMalloc(&L.cci, sizeof(unsigned short) * (cc.size() + 8));
    hipMemcpy(L.cci, cc.data(), sizeof(unsigned short) * cc.size(), hipMemcpyHostToDevice);
    hipMalloc(&L.cv, sizeof(double) * (vv.size() + 8));
    hipMemcpy(L.cv, vv.data(), sizeof(double) * vv.size(), hipMemcpyHostToDevice);
    return &L;
}

static Merged *mg_get(int slot, int G)
{
    Merged &M = D.mg[slot];
    if (M.G) return &M;
    const int n = D.n, ng = (n + G - 1) / G;
    const int *rp = D.hrp.data(), *ci = D.hci.data();
    if (n >= (1 << 27)) return nullptr;
    std::vector<int> gp(ng + 1);
    std::vector<unsigned> mk(D.nnz);
    std::vector<double> mv(D.nnz);
    std::vector<int> idx;
    for (int g = 0; g < ng; ++g) {
        const int r0 = g * G, r1 = std::min(n, r0 + G), a = rp[r0], e = rp[r1];
        gp[g] = a;
        idx.resize(e - a);
        for (int t = 0; t < e - a; ++t) idx[t] = a + t;
        std::stable_sort(idx.begin(), idx.end(), [&](int p, int q) { return ci[p] < ci[q]; });
        int r = r0;
        std::vector<int> rowof(e - a);
        for (int k = a; k < e; ++k) {
            while (rp[r + 1] <= k) ++r;
            rowof[k - a] = r - r0;
        }
        for (int t = 0; t < e - a; ++t) {
            mk[a + t] = ((unsigned)ci[idx[t]] << 5) | (unsigned)rowof[idx[t] - a];
            mv[a + t] = D.hv[idx[t]];
        }
    }
    gp[ng] = rp[n];
    M.G = G;
    hipMalloc(&M.gp, sizeof(int) * gp.size());
    hipMemcpy(M.gp, gp.data(), sizeof(int) * gp.size(), hipMemcpyHostToDevice);
    hipMalloc(&M.mk, sizeof(unsigned) * (mk.size() + 8));
    hipMemcpy(M.mk, mk.data(), sizeof(unsigned) * mk.size(), hipMemcpyHostToDevice);
    hipMalloc(&M.mv, sizeof(double) * (mv.size() + 8));
    hipMemcpy(M.mv, mv.data(), sizeof(double) * mv.size(), hipMemcpyHostToDevice);
    return &M;
}

template <int G, int U>
static void launch_mg(int slot)
{
    Merged *M = mg_get(slot, G);
    if (!M) return;
    const int ng = (D.n + G - 1) / G;
    hipLaunchKernelGGL((k_merged<G, U>), dim3((ng + 3) / 4), dim3(kB), 0, 0, D.n, M->gp, M->mk, M->mv, D.x, D.b, D.y);
}

template <int K, int NT, int R, int Q>
static void launch_lx(int slot, int nb)
{
    Lx *L = lx_get(slot, K, nb);
    if (!L) {
        fprintf(stderr, "lx_get(%d) failed\n", K);
        return;
    }
    hipLaunchKernelGGL((k_ldsx<K, NT, R, Q>), dim3(L->nb), dim3(NT), 0, 0, D.n, L->nchunk, L->rs, L->crp, L->cci,
                       L->cv, D.x, D.b, D.y);
}

template <int G, int U>
static void launch_vec(bool sorted)
{
    if (sorted) row_sorted();
    hipLaunchKernelGGL((k_vec<G, U>), dim3((D.n + kB / G - 1) / (kB / G)), dim3(kB), 0, 0, D.n, D.rp,
                       sorted ? D.rci : D.ci, sorted ? D.rv : D.v, D.x, D.b, D.y);
}

static SortedCfg *sorted_cfg(int T, int NT)
{
    const int slot = __builtin_ctz(T) - 11;
    SortedCfg &c = D.cfg[slot];
    if (c.T) return c.T == T && c.NT == NT ? &c : nullptr;
    const int n = D.n, sh = __builtin_ctz(T);
    if ((long long)n << sh > 0xffffffffLL) return nullptr;
    const int *rp = D.hrp.data(), *ci = D.hci.data();
    std::vector<int> blk;
    for (int r = 0; r < n;) {
        blk.push_back(r);
        int e = r + 1;
        if (rp[e] - rp[r] <= T)
            while (e < n && e - r < NT && rp[e + 1] - rp[r] <= T) ++e;
        r = e;
    }
    blk.push_back(n);
    std::vector<unsigned> pk(D.nnz);
    std::vector<double> vs(D.nnz);
    std::vector<int> idx;
    for (size_t bI = 0; bI + 1 < blk.size(); ++bI) {
        const int a0 = rp[blk[bI]], e0 = rp[blk[bI + 1]];
        for (int a = a0; a < e0; a += T) {
            const int e = std::min(e0, a + T);
            idx.resize(e - a);
            for (int t = 0; t < e - a; ++t) idx[t] = a + t;
            std::stable_sort(idx.begin(), idx.end(), [&](int p, int q) { return ci[p] < ci[q]; });
            for (int t = 0; t < e - a; ++t) pk[a + t] = ((unsigned)ci[idx[t]] << sh) | (unsigned)(idx[t] - a), vs[a + t] = D.hv[idx[t]];
        }
    }
    c.T = T, c.NT = NT, c.nblk = (int)blk.size() - 1;
    hipMalloc(&c.blk, sizeof(int) * blk.size());
    hipMemcpy(c.blk, blk.data(), sizeof(int) * blk.size(), hipMemcpyHostToDevice);
    hipMalloc(&c.pk, sizeof(unsigned) * pk.size());
    hipMemcpy(c.pk, pk.data(), sizeof(unsigned) * pk.size(), hipMemcpyHostToDevice);
    hipMalloc(&c.v, sizeof(double) * vs.size());
    hipMemcpy(c.v, vs.data(), sizeof(double) * vs.size(), hipMemcpyHostToDevice);
    return &c;
}

template <int T, int NT, bool NOLOAD = false>
static void launch_ts()
{
    SortedCfg *c = sorted_cfg(T, NT);
    if (!c) return;
    hipLaunchKernelGGL((k_tsort<T, NT, NOLOAD>), dim3(c->nblk), dim3(NT), 0, 0, c->blk, D.rp, c->pk, c->v, D.x, D.b, D.y);
}

static void launch(int variant)
{
    const int nw = (D.n + 3) / 4;
    switch (variant) {
    case 0: hipLaunchKernelGGL(k_tile<false>, dim3(D.nblk), dim3(kB), 0, 0, D.blk, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 1: hipLaunchKernelGGL(k_wave<256>, dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 2: hipLaunchKernelGGL(k_wave<512>, dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 3: hipLaunchKernelGGL(k_wave<1024>, dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 4: hipLaunchKernelGGL(k_wave_db<256>, dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 5: hipLaunchKernelGGL(k_wave_db<512>, dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 6: hipLaunchKernelGGL(k_mrow<4>, dim3((D.n + 15) / 16), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 7: hipLaunchKernelGGL(k_mrow<8>, dim3((D.n + 31) / 32), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 8: hipLaunchKernelGGL(k_mrow<16>, dim3((D.n + 63) / 64), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 9: hipLaunchKernelGGL(k_mrow<32>, dim3((D.n + 127) / 128), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 10: hipLaunchKernelGGL((k_lanerow<16, false>), dim3((D.n + 255) / 256), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 11: hipLaunchKernelGGL((k_lanerow<16, true>), dim3((D.n + 255) / 256), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 12: hipLaunchKernelGGL((k_lanerow<8, true>), dim3((D.n + 255) / 256), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 13: hipLaunchKernelGGL((k_lanerow<32, true>), dim3((D.n + 255) / 256), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 14: hipLaunchKernelGGL(k_tile<true>, dim3(D.nblk), dim3(kB), 0, 0, D.blk, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 15: hipLaunchKernelGGL((k_wave_db<256, true>), dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 16: hipLaunchKernelGGL((k_wave_db<512, true>), dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 17: hipLaunchKernelGGL((k_wave_db<1024, true>), dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.ci, D.v, D.x, D.b, D.y); break;
    case 18: if (D.pk11) hipLaunchKernelGGL(k_tile_sorted<false>, dim3(D.nblk), dim3(kB), 0, 0, D.blk, D.rp, D.pk11, D.v11, D.x, D.b, D.y); break;
    case 19: if (D.pk8) hipLaunchKernelGGL(k_wave_sorted, dim3(nw), dim3(kB), 0, 0, D.n, D.rp, D.pk8, D.v8, D.x, D.b, D.y); break;
    case 20: launch_ts<2048, 256>(); break;
    case 21: launch_ts<4096, 256>(); break;
    case 22: launch_ts<8192, 512>(); break;
    case 23: launch_ts<8192, 1024>(); break;
    case 24: launch_ts<16384, 1024>(); break;
    case 25: launch_ts<2048, 256, true>(); break;
    case 26: launch_vec<8, 4>(false); break;
    case 27: launch_vec<8, 4>(true); break;
    case 28: launch_vec<16, 4>(true); break;
    case 29: launch_vec<32, 4>(true); break;
    case 30: launch_vec<64, 4>(true); break;
    case 31: launch_vec<64, 4>(false); break;
    case 32: launch_vec<4, 4>(true); break;
    case 33: launch_vec<64, 8>(true); break;
    case 34: launch_lx<8192, 512, 4, 2>(0, 512); break;
    case 35: launch_lx<8192, 1024, 4, 2>(0, 512); break;
    case 36: launch_lx<16384, 1024, 4, 2>(1, 256); break;
    case 37: launch_lx<16384, 1024, 2, 4>(1, 256); break;
    case 38: launch_lx<16384, 1024, 8, 1>(1, 256); break;
    case 39: launch_lx<16384, 512, 4, 2>(1, 256); break;
    case 40: launch_mg<4, 4>(0); break;
    case 41: launch_mg<8, 4>(1); break;
    case 42: launch_mg<16, 4>(2); break;
    case 43: launch_mg<8, 2>(1); break;
    case 44: { Merged *M = mg_get(2, 16); if (M) hipLaunchKernelGGL(k_mlds<16>, dim3((D.n + 15) / 16), dim3(kB), 0, 0, D.n, M->gp, M->mk, M->mv, D.x, D.b, D.y); } break;
    case 45: { Merged *M = mg_get(3, 32); if (M) hipLaunchKernelGGL(k_mlds<32>, dim3((D.n + 31) / 32), dim3(kB), 0, 0, D.n, M->gp, M->mk, M->mv, D.x, D.b, D.y); } break;
    case 46: { Merged *M = mg_get(1, 8); if (M) hipLaunchKernelGGL(k_mlds<8>, dim3((D.n + 7) / 8), dim3(kB), 0, 0, D.n, M->gp, M->mk, M->mv, D.x, D.b, D.y); } break;
    default: break;
    }
}

// returns avg ms; copies y to host
extern "C" double lab_time(int variant, int reps, double *y_out)
{
    hipMemset(D.y, 0, sizeof(double) * D.n);
    (void)hipGetLastError();
    launch(variant);
    hipError_t le = hipGetLastError(), se = hipDeviceSynchronize();
    if (le != hipSuccess || se != hipSuccess)
        fprintf(stderr, "variant %d: launch %s, sync %s\n", variant, hipGetErrorString(le), hipGetErrorString(se));
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
