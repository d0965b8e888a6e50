// ell_lab.hip — level-0 dictionary-ELL residual variants on a 7-pt 400^3 operator (lab only).
//
// Measures y = b - A x with A in the engine's dictionary ELL layout (8 one-byte codes per row,
// per-block offset/value dictionaries) for launch/dependency variants, beside two floors: a pure
// stream of the same vector bytes, and the matrix-free stencil gather.  Not product code.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/ell_lab.hip -o tools/ell_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

constexpr int B = 256;

struct Smem {
    int dd[32];
    double vd[8];
};

__device__ __forceinline__ void load8(const unsigned char *ell, int r, unsigned &a, unsigned &b)
{
    const uint2 q = *reinterpret_cast<const uint2 *>(ell + (size_t)r * 8);
    a = q.x, b = q.y;
}
__device__ __forceinline__ void load8_nt(const unsigned char *ell, int r, unsigned &a, unsigned &b)
{
    const unsigned long long q = __builtin_nontemporal_load(reinterpret_cast<const unsigned long long *>(ell) + r);
    a = (unsigned)q, b = (unsigned)(q >> 32);
}
__device__ __forceinline__ double row_sum(unsigned w0, unsigned w1, int r, const Smem &s, const double *x)
{
    int c[8];
    double a[8], p[8];
    int len = 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const unsigned byte = ((k < 4 ? w0 : w1) >> (8 * (k & 3))) & 0xffu;
        if (byte == 0xffu && len == 8) len = k;
        c[k] = r + s.dd[byte & 31u];
        a[k] = s.vd[byte >> 5];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) p[k] = k < len ? a[k] * x[c[k]] : 0.0;
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (k < len) t += p[k];
    return t;
}

// A: the engine's current shape (block bounds loaded, dictionaries through pd)
template <int RPT>
__global__ __launch_bounds__(B) void kA(const int2 *blk, const int4 *pd, const int *dd, const double *vd,
                                        const unsigned char *ell, const double *x, const double *b, double *y, int nb)
{
    __shared__ Smem es[RPT];
    unsigned w0[RPT], w1[RPT];
    double br[RPT];
    int r[RPT];
    bool live[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int bid = blockIdx.x * RPT + j;
        live[j] = false;
        w0[j] = w1[j] = 0;
        br[j] = 0;
        r[j] = 0;
        if (bid < nb) {
            const int2 ba = blk[bid], be = blk[bid + 1];
            r[j] = ba.x + threadIdx.x;
            live[j] = r[j] < be.x;
            if (live[j]) load8(ell, r[j], w0[j], w1[j]), br[j] = b[r[j]];
            const int4 p = pd[bid];
            if ((int)threadIdx.x < p.y) es[j].dd[threadIdx.x] = dd[p.x + threadIdx.x];
            if ((int)threadIdx.x < p.w) es[j].vd[threadIdx.x] = vd[p.z + threadIdx.x];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RPT; ++j)
        if (live[j]) y[r[j]] = br[j] - row_sum(w0[j], w1[j], r[j], es[j], x);
}

// B: uniform 256-row blocks (row = block * 256 + thread), dictionaries at a fixed stride
// (32 offsets, 8 values per block): every load of the row issued at once, one barrier.
template <int RPT, bool NT>
__global__ __launch_bounds__(B) void kB(const int *ddf, const double *vdf, const unsigned char *ell, const double *x,
                                        const double *b, double *y, int n)
{
    __shared__ Smem es[RPT];
    unsigned w0[RPT], w1[RPT];
    double br[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int bid = blockIdx.x * RPT + j;
        const int r = bid * B + threadIdx.x;
        w0[j] = w1[j] = 0;
        br[j] = 0;
        if (r < n) {
            if (NT) load8_nt(ell, r, w0[j], w1[j]), br[j] = __builtin_nontemporal_load(b + r);
            else load8(ell, r, w0[j], w1[j]), br[j] = b[r];
        }
        if (threadIdx.x < 32) es[j].dd[threadIdx.x] = ddf[(size_t)bid * 32 + threadIdx.x];
        else if (threadIdx.x < 40) es[j].vd[threadIdx.x - 32] = vdf[(size_t)bid * 8 + threadIdx.x - 32];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int r = (blockIdx.x * RPT + j) * B + threadIdx.x;
        if (r < n) {
            const double v = br[j] - row_sum(w0[j], w1[j], r, es[j], x);
            if (NT) __builtin_nontemporal_store(v, y + r);
            else y[r] = v;
        }
    }
}

// D: dictionaries read straight from global memory (no LDS, no barrier): codes -> dictionary
// entries -> x.
template <int RPT>
__global__ __launch_bounds__(B) void kD(const int *ddf, const double *vdf, const unsigned char *ell, const double *x,
                                        const double *b, double *y, int n)
{
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int bid = blockIdx.x * RPT + j;
        const int r = bid * B + threadIdx.x;
        if (r >= n) continue;
        unsigned w0, w1;
        load8(ell, r, w0, w1);
        const double br = b[r];
        const int *dd = ddf + (size_t)bid * 32;
        const double *vd = vdf + (size_t)bid * 8;
        int c[8];
        double a[8];
        int len = 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const unsigned byte = ((k < 4 ? w0 : w1) >> (8 * (k & 3))) & 0xffu;
            if (byte == 0xffu && len == 8) len = k;
            c[k] = byte == 0xffu ? r : r + dd[byte & 31u];
            a[k] = byte == 0xffu ? 0.0 : vd[byte >> 5];
        }
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (k < len) t += a[k] * x[c[k]];
        y[r] = br - t;
    }
}

// F: persistent workgroups over the blocks, the next block's codes / b / dictionaries loaded
// while the current block gathers.
__global__ __launch_bounds__(B) void kF(const int *ddf, const double *vdf, const unsigned char *ell, const double *x,
                                        const double *b, double *y, int n, int nb)
{
    __shared__ Smem es[2];
    int bid = blockIdx.x;
    unsigned w0 = 0, w1 = 0;
    double br = 0;
    auto issue = [&](int q, int slot) {
        const int r = q * B + threadIdx.x;
        if (r < n) load8(ell, r, w0, w1), br = b[r];
        if (threadIdx.x < 32) es[slot].dd[threadIdx.x] = ddf[(size_t)q * 32 + threadIdx.x];
        else if (threadIdx.x < 40) es[slot].vd[threadIdx.x - 32] = vdf[(size_t)q * 8 + threadIdx.x - 32];
    };
    int slot = 0;
    if (bid < nb) issue(bid, 0);
    for (; bid < nb; bid += gridDim.x) {
        __syncthreads();
        const unsigned c0 = w0, c1 = w1;
        const double bb = br;
        const int nx = bid + gridDim.x;
        const int r = bid * B + threadIdx.x;
        if (nx < nb) issue(nx, slot ^ 1);
        if (r < n) y[r] = bb - row_sum(c0, c1, r, es[slot], x);
        slot ^= 1;
    }
}


__device__ __forceinline__ int xcd_remap(int b, int nb)
{
    const int per = nb >> 3, rem = nb & 7, xcd = b & 7, idx = b >> 3;
    return xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
}
// W: walkers.  Blocks form a (plane, tile) grid of stride S blocks; walker (tile t, chunk c) takes
// RPT consecutive blocks of each plane in [c * spc, (c + 1) * spc), one plane after the other, the
// next plane's codes / b / dictionaries loaded while the current one gathers.  Walkers of
// neighbouring tiles share an XCD (remap), so the x lines of the planes above and below are still
// in that XCD's L2 when the walker reaches them.
template <int RPT>
__global__ __launch_bounds__(B) void kW(const int *ddf, const double *vdf, const unsigned char *ell, const double *x,
                                        const double *b, double *y, int n, int nb, int S, int T, int spc, int remap)
{
    __shared__ Smem es[2][RPT];
    const int L = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int t = L % T, c = L / T;
    const int s0 = c * spc, s1 = s0 + spc;
    unsigned w0[RPT], w1[RPT];
    double br[RPT];
    auto issue = [&](int step, int slot) {
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
            const int q = t * RPT + j, bid = q + S * step;
            const int r = bid * B + threadIdx.x;
            w0[j] = w1[j] = 0xffffffffu;
            br[j] = 0.0;
            if (q < S && bid < nb) {
                if (r < n) load8(ell, r, w0[j], w1[j]), br[j] = b[r];
                if (threadIdx.x < 32) es[slot][j].dd[threadIdx.x] = ddf[(size_t)bid * 32 + threadIdx.x];
                else if (threadIdx.x < 40) es[slot][j].vd[threadIdx.x - 32] = vdf[(size_t)bid * 8 + threadIdx.x - 32];
            }
        }
    };
    int slot = 0;
    issue(s0, 0);
    for (int step = s0; step < s1; ++step) {
        __syncthreads();
        unsigned c0[RPT], c1[RPT];
        double bb[RPT];
#pragma unroll
        for (int j = 0; j < RPT; ++j) c0[j] = w0[j], c1[j] = w1[j], bb[j] = br[j];
        if (step + 1 < s1) issue(step + 1, slot ^ 1);
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
            const int q = t * RPT + j, bid = q + S * step;
            const int r = bid * B + threadIdx.x;
            if (q < S && bid < nb && r < n) y[r] = bb[j] - row_sum(c0[j], c1[j], r, es[slot][j], x);
        }
        slot ^= 1;
    }
}
// MW: the matrix-free stencil in the walker order (floor of the walk)
__global__ __launch_bounds__(B) void kMW(int N, const double *x, const double *b, double *y, int n, int nb, int S,
                                         int T, int spc, int remap, int RPT)
{
    const int L = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int t = L % T, c = L / T;
    for (int step = c * spc; step < (c + 1) * spc; ++step)
        for (int j = 0; j < RPT; ++j) {
            const int q = t * RPT + j, bid = q + S * step;
            const int r = bid * B + threadIdx.x;
            if (q >= S || bid >= nb || r >= n) continue;
            const int i = r % N, jj = (r / N) % N, k = r / (N * N);
            double tt = 6.0 * x[r];
            if (k > 0) tt -= x[r - N * N];
            if (jj > 0) tt -= x[r - N];
            if (i > 0) tt -= x[r - 1];
            if (i < N - 1) tt -= x[r + 1];
            if (jj < N - 1) tt -= x[r + N];
            if (k < N - 1) tt -= x[r + N * N];
            y[r] = b[r] - tt;
        }
}


// probes of the memory pipeline: Sd = 7 loads of the same x[r] (L1 hits), Sf = 7 loads of far,
// distinct x lines (no reuse), both + b + y
__global__ __launch_bounds__(B) void kSd(const double *x, const double *b, double *y, int n)
{
    const int r = blockIdx.x * B + threadIdx.x;
    if (r >= n) return;
    const volatile double *xv = x;
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k) t += xv[r];
    y[r] = b[r] - t;
}
__global__ __launch_bounds__(B) void kSf(int NN, const double *x, const double *b, double *y, int n)
{
    const int r = blockIdx.x * B + threadIdx.x;
    if (r >= n) return;
    double t = 0.0;
#pragma unroll
    for (int k = -3; k <= 3; ++k) {
        long long c = (long long)r + (long long)k * NN;
        if (c < 0) c += n;
        if (c >= n) c -= n;
        t += x[c];
    }
    y[r] = b[r] - t;
}
// ML: matrix-free with x[r0 - N, r1 + N) staged in LDS (16-byte loads), the +-N^2 planes from global
__global__ __launch_bounds__(B) void kML(int N, const double *x, const double *b, double *y, int n)
{
    extern __shared__ double win[];
    const int r0 = blockIdx.x * B, lo = r0 - N, cnt = B + 2 * N;
    for (int t = 2 * threadIdx.x; t < cnt; t += 2 * B) {
        const int g = lo + t;
        if (g >= 0 && g + 1 < n && ((g & 1) == 0)) {
            const double2 q = *reinterpret_cast<const double2 *>(x + g);
            win[t] = q.x, win[t + 1] = q.y;
        } else {
            if (g >= 0 && g < n) win[t] = x[g];
            if (t + 1 < cnt && g + 1 >= 0 && g + 1 < n) win[t + 1] = x[g + 1];
        }
    }
    const int r = r0 + threadIdx.x;
    double xm = 0, xp = 0, br = 0;
    const int i = r % N, j = (r / N) % N, k = r / (N * N);
    if (r < n) {
        br = b[r];
        if (k > 0) xm = x[r - N * N];
        if (k < N - 1) xp = x[r + N * N];
    }
    __syncthreads();
    if (r >= n) return;
    const double *w = win + (r - lo);
    double t = 6.0 * w[0];
    if (k > 0) t -= xm;
    if (j > 0) t -= w[-N];
    if (i > 0) t -= w[-1];
    if (i < N - 1) t -= w[1];
    if (j < N - 1) t -= w[N];
    if (k < N - 1) t -= xp;
    y[r] = b[r] - t;
}
// EL: dictionary ELL with offsets |off| <= WIN served from an LDS window of x (launch parameter)
template <int RPT>
__global__ __launch_bounds__(B) void kEL(const int *ddf, const double *vdf, const unsigned char *ell, const double *x,
                                         const double *b, double *y, int n, int WIN)
{
    extern __shared__ double win[];
    __shared__ Smem es[RPT];
    const int r0 = blockIdx.x * RPT * B, lo = r0 - WIN, cnt = RPT * B + 2 * WIN;
    unsigned w0[RPT], w1[RPT];
    double br[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int bid = blockIdx.x * RPT + j;
        const int r = bid * B + threadIdx.x;
        w0[j] = w1[j] = 0xffffffffu;
        br[j] = 0;
        if (r < n) load8(ell, r, w0[j], w1[j]), br[j] = b[r];
        if (threadIdx.x < 32) es[j].dd[threadIdx.x] = ddf[(size_t)bid * 32 + threadIdx.x];
        else if (threadIdx.x < 40) es[j].vd[threadIdx.x - 32] = vdf[(size_t)bid * 8 + threadIdx.x - 32];
    }
    for (int t = 2 * threadIdx.x; t < cnt; t += 2 * B) {
        const int g = lo + t;   // lo even (r0, WIN even)
        if (g >= 0 && g + 1 < n) {
            const double2 q = *reinterpret_cast<const double2 *>(x + g);
            win[t] = q.x, win[t + 1] = q.y;
        } else if (g >= 0 && g < n) {
            win[t] = x[g];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int r = (blockIdx.x * RPT + j) * B + threadIdx.x;
        if (r >= n) continue;
        int c[8];
        double a[8], p[8];
        int len = 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const unsigned byte = ((k < 4 ? w0[j] : w1[j]) >> (8 * (k & 3))) & 0xffu;
            if (byte == 0xffu && len == 8) len = k;
            c[k] = es[j].dd[byte & 31u];
            a[k] = es[j].vd[byte >> 5];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            double xv = 0.0;
            if (k < len) xv = (c[k] >= -WIN && c[k] <= WIN) ? win[r - lo + c[k]] : x[r + c[k]];
            p[k] = k < len ? a[k] * xv : 0.0;
        }
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (k < len) t += p[k];
        y[r] = br[j] - t;
    }
}


// EW: walkers with an LDS ring of x windows.  Walker (tile t, chunk c) takes rows
// [t R + k P, t R + k P + R) of planes k in its chunk (R = RPT * 256, P = plane rows); x of
// [t R + j P - WX, t R + j P + R + WX) for planes j = k - 1, k, k + 1 sits in ring slots j % 4, the
// window of plane k + 2 is loaded during step k.  An offset o is served from the window of plane
// k + m, m = the nearest multiple of P, when it falls inside it; else from global x.
template <int RPT>
__global__ __launch_bounds__(B) void kEW(const int *ddf, const double *vdf, const unsigned char *ell, const double *x,
                                         const double *b, double *y, int n, int P, int T, int spc, int WX)
{
    extern __shared__ double ring[];   // 4 slots of (R + 2 WX) doubles
    __shared__ Smem es[2][RPT];
    constexpr int R = RPT * B;
    const int WL = R + 2 * WX;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int t = L % T, c = L / T;
    const int nplanes = (n + P - 1) / P;
    const int k0 = c * spc, k1 = min(nplanes, k0 + spc);
    if (k0 >= k1) return;
    auto load_win = [&](int j) {   // window of plane j into slot j & 3 (16-byte loads)
        double *w = ring + (size_t)(j & 3) * WL;
        const int g0 = t * R + j * P - WX;   // even (R, P, WX even)
        for (int q = 2 * threadIdx.x; q < WL; q += 2 * B) {
            const int g = g0 + q;
            double2 v = make_double2(0.0, 0.0);
            if (j >= 0 && j < nplanes && g >= 0 && g + 1 < n) v = *reinterpret_cast<const double2 *>(x + g);
            else if (j >= 0 && j < nplanes && g >= 0 && g < n) v.x = x[g];
            w[q] = v.x;
            if (q + 1 < WL) w[q + 1] = v.y;
        }
    };
    unsigned w0[RPT], w1[RPT];
    double br[RPT];
    auto issue = [&](int k, int slot) {
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
            const int base = t * R + k * P + j * B;
            const int r = base + threadIdx.x;
            const bool ok = t * R + j * B < P && r < n;
            w0[j] = w1[j] = 0xffffffffu;
            br[j] = 0.0;
            if (ok) load8(ell, r, w0[j], w1[j]), br[j] = b[r];
            const int bid = base / B;
            if (t * R + j * B < P && base < n) {
                if (threadIdx.x < 32) es[slot][j].dd[threadIdx.x] = ddf[(size_t)bid * 32 + threadIdx.x];
                else if (threadIdx.x < 40) es[slot][j].vd[threadIdx.x - 32] = vdf[(size_t)bid * 8 + threadIdx.x - 32];
            }
        }
    };
    load_win(k0 - 1);
    load_win(k0);
    load_win(k0 + 1);
    issue(k0, 0);
    int slot = 0;
    for (int k = k0; k < k1; ++k) {
        __syncthreads();   // windows k-1..k+1 and the dictionaries of step k in LDS
        unsigned c0[RPT], c1[RPT];
        double bb[RPT];
#pragma unroll
        for (int j = 0; j < RPT; ++j) c0[j] = w0[j], c1[j] = w1[j], bb[j] = br[j];
        if (k + 1 < k1) issue(k + 1, slot ^ 1);
        if (k + 2 < k1 + 1) load_win(k + 2);   // slot (k+2)&3 = (k-2)&3: no longer read
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
            const int r = t * R + k * P + j * B + threadIdx.x;
            if (!(t * R + j * B < P) || r >= n) continue;
            const int lr = j * B + threadIdx.x;   // row position inside the step's rows
            int o[8];
            double a[8], p[8];
            int len = 8;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const unsigned byte = ((q < 4 ? c0[j] : c1[j]) >> (8 * (q & 3))) & 0xffu;
                if (byte == 0xffu && len == 8) len = q;
                o[q] = es[slot][j].dd[byte & 31u];
                a[q] = es[slot][j].vd[byte >> 5];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                double xv = 0.0;
                if (q < len) {
                    const int m = o[q] > P / 2 ? 1 : (o[q] < -P / 2 ? -1 : 0);
                    const int loc = lr + o[q] - m * P + WX;
                    xv = (loc >= 0 && loc < WL) ? ring[(size_t)((k + m) & 3) * WL + loc] : x[r + o[q]];
                }
                p[q] = q < len ? a[q] * xv : 0.0;
            }
            double s = 0.0;
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (q < len) s += p[q];
            y[r] = bb[j] - s;
        }
        slot ^= 1;
    }
}

// floors: S streams codes, b, x (coalesced), writes y; M is the matrix-free 7-pt residual
__global__ __launch_bounds__(B) void kS(const unsigned char *ell, const double *x, const double *b, double *y, int n)
{
    const int r = blockIdx.x * B + threadIdx.x;
    if (r >= n) return;
    unsigned w0, w1;
    load8(ell, r, w0, w1);
    y[r] = b[r] - x[r] * (double)(w0 ^ w1);
}
__global__ __launch_bounds__(B) void kM(int N, const double *x, const double *b, double *y, int n)
{
    const int r = blockIdx.x * B + threadIdx.x;
    if (r >= n) return;
    const int i = r % N, j = (r / N) % N, k = r / (N * N);
    double t = 6.0 * x[r];
    if (k > 0) t -= x[r - N * N];
    if (j > 0) t -= x[r - N];
    if (i > 0) t -= x[r - 1];
    if (i < N - 1) t -= x[r + 1];
    if (j < N - 1) t -= x[r + N];
    if (k < N - 1) t -= x[r + N * N];
    y[r] = b[r] - t;
}

int main(int argc, char **argv)
{
    const int N = argc > 1 ? atoi(argv[1]) : 400;
    const int n = N * N * N, nb = (n + B - 1) / B;
    const int offs[7] = {-N * N, -N, -1, 0, 1, N, N * N};
    std::vector<unsigned char> ell((size_t)n * 8, 0xff);
    std::vector<int> ddf((size_t)nb * 32, 0);
    std::vector<double> vdf((size_t)nb * 8, 0.0);
    std::vector<int4> pd(nb);
    std::vector<int2> blk(nb + 1);
    std::vector<int> dd;
    std::vector<double> vd;
    for (int q = 0; q < nb; ++q) {
        pd[q] = make_int4((int)dd.size(), 7, (int)vd.size(), 2);
        for (int t = 0; t < 7; ++t) dd.push_back(offs[t]), ddf[(size_t)q * 32 + t] = offs[t];
        vd.push_back(-1.0), vd.push_back(6.0);
        vdf[(size_t)q * 8] = -1.0, vdf[(size_t)q * 8 + 1] = 6.0;
        blk[q] = make_int2(q * B, 0);
    }
    blk[nb] = make_int2(n, 0);
    for (int r = 0; r < n; ++r) {
        const int i = r % N, j = (r / N) % N, k = r / (N * N);
        const bool in[7] = {k > 0, j > 0, i > 0, true, i < N - 1, j < N - 1, k < N - 1};
        int s = 0;
        for (int t = 0; t < 7; ++t)
            if (in[t]) ell[(size_t)r * 8 + s++] = (unsigned char)((t == 3 ? 1 : 0) << 5 | t);
    }
    unsigned char *d_ell;
    int *d_ddf, *d_dd;
    double *d_vdf, *d_vd, *x, *b, *y, *y0;
    int4 *d_pd;
    int2 *d_blk;
    CK(hipMalloc(&d_ell, ell.size()));
    CK(hipMalloc(&d_ddf, ddf.size() * 4));
    CK(hipMalloc(&d_vdf, vdf.size() * 8));
    CK(hipMalloc(&d_dd, dd.size() * 4));
    CK(hipMalloc(&d_vd, vd.size() * 8));
    CK(hipMalloc(&d_pd, pd.size() * 16));
    CK(hipMalloc(&d_blk, blk.size() * 8));
    CK(hipMalloc(&x, (size_t)n * 8));
    CK(hipMalloc(&b, (size_t)n * 8));
    CK(hipMalloc(&y, (size_t)n * 8));
    CK(hipMalloc(&y0, (size_t)n * 8));
    CK(hipMemcpy(d_ell, ell.data(), ell.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ddf, ddf.data(), ddf.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_vdf, vdf.data(), vdf.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_dd, dd.data(), dd.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_vd, vd.data(), vd.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_pd, pd.data(), pd.size() * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_blk, blk.data(), blk.size() * 8, hipMemcpyHostToDevice));
    {
        std::vector<double> h(n);
        for (int r = 0; r < n; ++r) h[r] = 1.0 + 1e-3 * (r % 977);
        CK(hipMemcpy(x, h.data(), (size_t)n * 8, hipMemcpyHostToDevice));
        for (int r = 0; r < n; ++r) h[r] = 1.0 - 1e-3 * (r % 331);
        CK(hipMemcpy(b, h.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    }
    int ncu = 256;
    {
        hipDeviceProp_t p;
        CK(hipGetDeviceProperties(&p, 0));
        ncu = p.multiProcessorCount;
    }
    const double bytes = 8.0 * n + 24.0 * n + 16.0 * nb + 4.0 * 7 * nb + 8.0 * 2 * nb + 8.0 * nb;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> ref(n), got(n);
    auto run = [&](const char *name, auto launch, bool check) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        bool ok = true;
        if (check) {
            CK(hipMemcpy(got.data(), y, (size_t)n * 8, hipMemcpyDeviceToHost));
            ok = memcmp(got.data(), ref.data(), (size_t)n * 8) == 0;
        }
        printf("%-28s %8.1f us  %7.0f GB/s (%4.1f%% of 8 TB/s)%s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
               100.0 * bytes / (ms * 1e-3) / 8e12, check ? (ok ? "  bitwise" : "  MISMATCH") : "");
        fflush(stdout);
    };
    run("A rpt1 (engine shape)", [&] { hipLaunchKernelGGL(kA<1>, dim3(nb), dim3(B), 0, 0, d_blk, d_pd, d_dd, d_vd, d_ell, x, b, y, nb); }, false);
    CK(hipMemcpy(ref.data(), y, (size_t)n * 8, hipMemcpyDeviceToHost));
    run("A rpt2 (engine HEAD)", [&] { hipLaunchKernelGGL(kA<2>, dim3((nb + 1) / 2), dim3(B), 0, 0, d_blk, d_pd, d_dd, d_vd, d_ell, x, b, y, nb); }, true);
    run("B rpt1 implicit/fixed", [&] { hipLaunchKernelGGL((kB<1, false>), dim3(nb), dim3(B), 0, 0, d_ddf, d_vdf, d_ell, x, b, y, n); }, true);
    run("B rpt2", [&] { hipLaunchKernelGGL((kB<2, false>), dim3((nb + 1) / 2), dim3(B), 0, 0, d_ddf, d_vdf, d_ell, x, b, y, n); }, true);
    run("B rpt4", [&] { hipLaunchKernelGGL((kB<4, false>), dim3((nb + 3) / 4), dim3(B), 0, 0, d_ddf, d_vdf, d_ell, x, b, y, n); }, true);
    run("G rpt1 nontemporal", [&] { hipLaunchKernelGGL((kB<1, true>), dim3(nb), dim3(B), 0, 0, d_ddf, d_vdf, d_ell, x, b, y, n); }, true);
    run("G rpt2 nontemporal", [&] { hipLaunchKernelGGL((kB<2, true>), dim3((nb + 1) / 2), dim3(B), 0, 0, d_ddf, d_vdf, d_ell, x, b, y, n); }, true);
    run("D rpt1 global dicts", [&] { hipLaunchKernelGGL(kD<1>, dim3(nb), dim3(B), 0, 0, d_ddf, d_vdf, d_ell, x, b, y, n); }, true);
    run("D rpt2 global dicts", [&] { hipLaunchKernelGGL(kD<2>, dim3((nb + 1) / 2), dim3(B), 0, 0, d_ddf, d_vdf, d_ell, x, b, y, n); }, true);
    for (int m : {4, 8, 16}) {
        char nm[64];
        snprintf(nm, sizeof nm, "F persistent %dx CUs", m);
        run(nm, [&] { hipLaunchKernelGGL(kF, dim3(ncu * m), dim3(B), 0, 0, d_ddf, d_vdf, d_ell, x, b, y, n, nb); }, true);
    }

    run("Sd 7 same-address loads", [&] { hipLaunchKernelGGL(kSd, dim3(nb), dim3(B), 0, 0, x, b, y, n); }, false);
    run("Sf 7 far distinct loads", [&] { hipLaunchKernelGGL(kSf, dim3(nb), dim3(B), 0, 0, N * N, x, b, y, n); }, false);
    run("ML matrix-free LDS window", [&] { hipLaunchKernelGGL(kML, dim3(nb), dim3(B), (B + 2 * N + 2) * 8, 0, N, x, b, y, n); }, false);
    run("EL rpt1 LDS window", [&] { hipLaunchKernelGGL(kEL<1>, dim3(nb), dim3(B), (B + 2 * N + 2) * 8, 0, d_ddf, d_vdf, d_ell, x, b, y, n, N); }, true);
    run("EL rpt2 LDS window", [&] { hipLaunchKernelGGL(kEL<2>, dim3((nb + 1) / 2), dim3(B), (2 * B + 2 * N + 2) * 8, 0, d_ddf, d_vdf, d_ell, x, b, y, n, N); }, true);
    run("EL rpt4 LDS window", [&] { hipLaunchKernelGGL(kEL<4>, dim3((nb + 3) / 4), dim3(B), (4 * B + 2 * N + 2) * 8, 0, d_ddf, d_vdf, d_ell, x, b, y, n, N); }, true);

    for (int rpt : {1, 2, 4})
        for (int C : {8, 16, 40}) {
            const int P = N * N, R = rpt * B, T = (P + R - 1) / R, spc = (N + C - 1) / C, G = T * C;
            const size_t lds = 4 * (size_t)(R + 2 * N) * 8;
            char nm[64];
            snprintf(nm, sizeof nm, "EW rpt%d chunks%d", rpt, C);
            if (rpt == 1) run(nm, [&] { hipLaunchKernelGGL(kEW<1>, dim3(G), dim3(B), lds, 0, d_ddf, d_vdf, d_ell, x, b, y, n, P, T, spc, N); }, true);
            if (rpt == 2) run(nm, [&] { hipLaunchKernelGGL(kEW<2>, dim3(G), dim3(B), lds, 0, d_ddf, d_vdf, d_ell, x, b, y, n, P, T, spc, N); }, true);
            if (rpt == 4) run(nm, [&] { hipLaunchKernelGGL(kEW<4>, dim3(G), dim3(B), lds, 0, d_ddf, d_vdf, d_ell, x, b, y, n, P, T, spc, N); }, true);
        }
    run("M matrix-free stencil", [&] { hipLaunchKernelGGL(kM, dim3(nb), dim3(B), 0, 0, N, x, b, y, n); }, false);
    run("S stream floor", [&] { hipLaunchKernelGGL(kS, dim3(nb), dim3(B), 0, 0, d_ell, x, b, y, n); }, false);
    return 0;
}
