// l0_lab.hip — level-0 kernels of the 7-pt 400^3 hierarchy, rows per thread (lab only, not product code).
//
// The level-0 operator as the engine stores it: rows relabeled F-first / C-second (red-black: F =
// odd points, C = even points), each row's stored-order entries as one-byte codes (value index << 5
// | offset index, 0xFF pads) into per-256-row-block dictionaries of column offsets (col - row) and
// values (sss_spmv_dev.hpp ell_decode).  Measures, for R = 1, 2, 4 consecutive rows per thread:
//   F pass : x_r = (b_r - sum_{s != diag} a_s x_{c_s}) / a_rr over the F rows (relax_range MODE 0)
//   resid  : y_r = b_r - sum_s a_s x_{c_s} over every row (spmv_adaptive RESID)
// R >= 2 gathers the x of two neighbouring rows with one 16-byte load where their columns are
// adjacent (c_{r+1,s} = c_{r,s} + 1: the same stencil offset); every row's sum keeps its stored order,
// so every variant is bitwise the R = 1 kernel (checked).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/l0_lab.hip -o tools/l0_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

constexpr int B = 256;   // rows per dictionary block

struct __attribute__((aligned(8))) D2 {
    double a, b;
};

template <int R>
struct Codes {
    unsigned w[2 * R];
};
template <int R>
__device__ __forceinline__ void load_codes(const unsigned char *ell, int r0, Codes<R> &c)
{
    if constexpr (R == 1) {
        const uint2 q = *reinterpret_cast<const uint2 *>(ell + (size_t)r0 * 8);
        c.w[0] = q.x, c.w[1] = q.y;
    } else {
#pragma unroll
        for (int h = 0; h < R / 2; ++h) {
            const uint4 q = *reinterpret_cast<const uint4 *>(ell + (size_t)r0 * 8 + 16 * h);
            c.w[4 * h] = q.x, c.w[4 * h + 1] = q.y, c.w[4 * h + 2] = q.z, c.w[4 * h + 3] = q.w;
        }
    }
}

// MODE 0: F pass (in place, diagonal product skipped, no fetch of x_r); MODE 1: residual.
// PAIR: pair loads for R >= 2.  Grid: one workgroup per R blocks of rows [lo, hi).
template <int MODE, int R, bool PAIR>
__global__ __launch_bounds__(B) void kpass(const unsigned char *__restrict__ ell, const int *__restrict__ ddf,
                                           const double *__restrict__ vdf, const double *__restrict__ b,
                                           double *x, double *__restrict__ y, int lo, int hi)
{
    __shared__ int dd[R][32];
    __shared__ double vd[R][8];
    const int blk0 = lo / B + blockIdx.x * R;
    if (threadIdx.x < 32 * R) {
        const int j = threadIdx.x >> 5, t = threadIdx.x & 31;
        dd[j][t] = ddf[(size_t)(blk0 + j) * 32 + t];
        if (t < 8) vd[j][t] = vdf[(size_t)(blk0 + j) * 8 + t];
    }
    const int r0 = lo + blockIdx.x * R * B + R * threadIdx.x;
    const bool live = r0 < hi;   // hi a multiple of R (checked on the host)
    Codes<R> cw;
    double br[R];
#pragma unroll
    for (int i = 0; i < 2 * R; ++i) cw.w[i] = 0xffffffffu;
#pragma unroll
    for (int i = 0; i < R; ++i) br[i] = 0.0;
    if (live) {
        load_codes<R>(ell, r0, cw);
        if constexpr (R == 1) br[0] = b[r0];
        else {
#pragma unroll
            for (int h = 0; h < R / 2; ++h) {
                const double2 q = *reinterpret_cast<const double2 *>(b + r0 + 2 * h);
                br[2 * h] = q.x, br[2 * h + 1] = q.y;
            }
        }
    }
    __syncthreads();
    if (!live) return;
    const int j = (R * threadIdx.x) / B;
    int c[R][8], len[R], ds[R];
    double a[R][8], dv[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        len[i] = 8;
        ds[i] = -1;
        dv[i] = 0.0;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const unsigned byte = (cw.w[2 * i + (s >> 2)] >> (8 * (s & 3))) & 0xffu;
            if (byte == 0xffu && len[i] == 8) len[i] = s;
            c[i][s] = r0 + i + dd[j][byte & 31u];
            a[i][s] = vd[j][byte >> 5];
        }
#pragma unroll
        for (int s = 0; s < 8; ++s)
            if (s < len[i] && c[i][s] == r0 + i) ds[i] = s, dv[i] = a[i][s];
    }
    double xv[R][8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        if constexpr (PAIR && R >= 2) {
#pragma unroll
            for (int i = 0; i < R; i += 2) {
                const bool n0 = s < len[i] && (MODE == 1 || s != ds[i]);
                const bool n1 = s < len[i + 1] && (MODE == 1 || s != ds[i + 1]);
                if (n0 && n1 && c[i + 1][s] == c[i][s] + 1) {
                    const D2 q = *reinterpret_cast<const D2 *>(x + c[i][s]);
                    xv[i][s] = q.a, xv[i + 1][s] = q.b;
                } else {
                    xv[i][s] = n0 ? x[c[i][s]] : 0.0;
                    xv[i + 1][s] = n1 ? x[c[i + 1][s]] : 0.0;
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < R; ++i)
                xv[i][s] = (s < len[i] && (MODE == 1 || s != ds[i])) ? x[c[i][s]] : 0.0;
        }
    }
    double out[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        if constexpr (MODE == 0) {
            double t = br[i];
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (s < len[i] && s != ds[i]) t -= a[i][s] * xv[i][s];
            out[i] = fabs(dv[i]) > 1e-20 ? t / dv[i] : x[r0 + i];
        } else {
            double t = 0.0;
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (s < len[i]) t += a[i][s] * xv[i][s];
            out[i] = br[i] + t * -1.0;
        }
    }
    double *dst = MODE == 0 ? x : y;
    if constexpr (R == 1) dst[r0] = out[0];
    else {
#pragma unroll
        for (int h = 0; h < R / 2; ++h)
            *reinterpret_cast<double2 *>(dst + r0 + 2 * h) = make_double2(out[2 * h], out[2 * h + 1]);
    }
}


// ---- persistent, software-pipelined pass (round 5 lab; measured and rejected) -------------------
// At 400^3: F pass 314-436 us for G = 4096..512 workgroups against 281 us for kpass<0, 1> (one block
// per workgroup); residual 654-811 us against 577 us.  The compiler branches around every gather and
// waits vmcnt(0) at the loop latch, so the next block's loads never overlap this block's gathers.
// (Run-coded dictionary ELL blocks -- codes stored once per run of equal rows, 2.1 GB fewer bytes per
// V-cycle -- measured in the engine the same round: level-0 smoothing 2112 -> 2301 us: the level-0
// passes are bound by each workgroup's chain of dependent loads, not by bytes.)
// Each workgroup loops over the blocks bq = blockIdx.x, + gridDim.x, ...  While block k's gathers are
// in flight, block k + 1's codes, b and dictionary values are loaded (registers), then stored to the
// other LDS dictionary buffer after block k's results: one barrier per block, and the dependent
// chain (dictionaries -> barrier -> decode -> gathers) of the next block overlaps this block's.
template <int MODE>
__global__ __launch_bounds__(B) void kpipe(const unsigned char *__restrict__ ell, const int *__restrict__ ddf,
                                           const double *__restrict__ vdf, const double *__restrict__ b,
                                           double *x, double *__restrict__ y, int lo, int hi)
{
    __shared__ int dd[2][32];
    __shared__ double vd[2][8];
    const int nb = (hi - lo + B - 1) / B, b0 = lo / B;
    int bq = blockIdx.x;
    if (bq >= nb) return;
    const int t = threadIdx.x;
    auto codes = [&](int q, unsigned (&w)[2], double &bv) {
        const int r = lo + q * B + t;
        w[0] = w[1] = 0xffffffffu;
        bv = 0.0;
        if (r < hi) {
            const uint2 c = *reinterpret_cast<const uint2 *>(ell + (size_t)r * 8);
            w[0] = c.x, w[1] = c.y;
            bv = b[r];
        }
    };
    int dreg = 0;
    double vreg = 0.0;
    auto dict_load = [&](int q) {
        if (t < 32) dreg = ddf[(size_t)(b0 + q) * 32 + t];
        else if (t < 40) vreg = vdf[(size_t)(b0 + q) * 8 + t - 32];
    };
    auto dict_store = [&](int buf) {
        if (t < 32) dd[buf][t] = dreg;
        else if (t < 40) vd[buf][t - 32] = vreg;
    };
    unsigned wc[2];
    double bc;
    codes(bq, wc, bc);
    dict_load(bq);
    dict_store(0);
    int buf = 0;
    for (;;) {
        __syncthreads();   // dictionaries of bq in dd[buf]; every reader of dd[buf ^ 1] is done
        const int r = lo + bq * B + t;
        const bool live = r < hi;
        int c[8], len = 8, ds = -1;
        double a[8], dv = 0.0;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const unsigned byte = (wc[s >> 2] >> (8 * (s & 3))) & 0xffu;
            if (byte == 0xffu && len == 8) len = s;
            c[s] = r + dd[buf][byte & 31u];
            a[s] = vd[buf][byte >> 5];
        }
#pragma unroll
        for (int s = 0; s < 8; ++s)
            if (s < len && c[s] == r) ds = s, dv = a[s];
        double xv[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) xv[s] = (live && s < len && (MODE == 1 || s != ds)) ? x[c[s]] : 0.0;
        const int nq = bq + gridDim.x;
        unsigned wn[2];
        double bn = 0.0;
        if (nq < nb) {   // the next block's loads, behind this block's gathers
            codes(nq, wn, bn);
            dict_load(nq);
        }
        if (live) {
            double out;
            if constexpr (MODE == 0) {
                double tt = bc;
#pragma unroll
                for (int s = 0; s < 8; ++s)
                    if (s < len && s != ds) tt -= a[s] * xv[s];
                out = fabs(dv) > 1e-20 ? tt / dv : x[r];
                x[r] = out;
            } else {
                double tt = 0.0;
#pragma unroll
                for (int s = 0; s < 8; ++s)
                    if (s < len) tt += a[s] * xv[s];
                y[r] = bc + tt * -1.0;
            }
        }
        if (nq >= nb) break;
        dict_store(buf ^ 1);
        buf ^= 1;
        bq = nq;
        wc[0] = wn[0], wc[1] = wn[1];
        bc = bn;
    }
}

// ---- x staged in LDS by offset ranges (round 5 lab; measured and rejected) --------------------------
// 7-pt 400^3 (profiles/r05_l0_lab_lds_stage.txt): 3-4 merged ranges, 1,167-1,423 staged doubles per
// block against 1,792 gathered values, yet the F pass took 487 us against 283 us and the residual 984
// against 574 us -- the range loads, the LDS stores and the second barrier lengthen each workgroup's
// chain of dependent steps, which is what bounds these kernels, and cut its occupancy.
// A 256-row block's rows read x at r + o for the block's few distinct offsets o; the host merges the
// intervals [r0 + o, r0 + o + 256) into at most SR ranges, which the workgroup loads coalesced into
// LDS; each entry then reads its x from LDS at lofs[d] + (r - r0) instead of a scattered gather.
constexpr int SR = 8, SBUD = 3072;   // ranges per block, staged doubles per block
struct StagePlan {
    int nr;                 // ranges (-1: not staged, gather)
    int gs[SR], len[SR], lb[SR];
    int lofs[32];           // per offset index: LDS position of row r0's value (-1: not staged)
};
template <int MODE>
__global__ __launch_bounds__(B) void kstage(const unsigned char *__restrict__ ell, const int *__restrict__ ddf,
                                            const double *__restrict__ vdf, const StagePlan *__restrict__ plan,
                                            const double *__restrict__ b, double *x, double *__restrict__ y, int lo, int hi)
{
    __shared__ int dd[32];
    __shared__ double vd[8];
    __shared__ StagePlan sp;
    __shared__ double xl[SBUD];
    const int blk = lo / B + blockIdx.x;
    const int t = threadIdx.x;
    if (t < 32) dd[t] = ddf[(size_t)blk * 32 + t];
    if (t < 8) vd[t] = vdf[(size_t)blk * 8 + t];
    {
        const int *src = reinterpret_cast<const int *>(plan + blk);
        int *dst = reinterpret_cast<int *>(&sp);
        constexpr int NW = sizeof(StagePlan) / 4;
        if (t < NW) dst[t] = src[t];
    }
    const int r = lo + blockIdx.x * B + t;
    const bool live = r < hi;
    unsigned w[2] = {0xffffffffu, 0xffffffffu};
    double br = 0.0;
    if (live) {
        const uint2 q = *reinterpret_cast<const uint2 *>(ell + (size_t)r * 8);
        w[0] = q.x, w[1] = q.y;
        br = b[r];
    }
    __syncthreads();
    const int nr = sp.nr;
    for (int k = 0; k < nr; ++k)   // coalesced range loads
        for (int e = t; e < sp.len[k]; e += B) xl[sp.lb[k] + e] = x[sp.gs[k] + e];
    __syncthreads();
    if (!live) return;
    int d[8], len = 8, ds = -1;
    double a[8], dv = 0.0;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const unsigned byte = (w[s >> 2] >> (8 * (s & 3))) & 0xffu;
        if (byte == 0xffu && len == 8) len = s;
        d[s] = byte & 31u;
        a[s] = vd[byte >> 5];
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
        if (s < len && dd[d[s]] == 0) ds = s, dv = a[s];
    double xv[8];
    const int tl = r - (lo + blockIdx.x * B);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const bool need = s < len && (MODE == 1 || s != ds);
        xv[s] = need ? (nr >= 0 ? xl[sp.lofs[d[s]] + tl] : x[r + dd[d[s]]]) : 0.0;
    }
    if constexpr (MODE == 0) {
        double tt = br;
#pragma unroll
        for (int s = 0; s < 8; ++s)
            if (s < len && s != ds) tt -= a[s] * xv[s];
        x[r] = fabs(dv) > 1e-20 ? tt / dv : x[r];
    } else {
        double tt = 0.0;
#pragma unroll
        for (int s = 0; s < 8; ++s)
            if (s < len) tt += a[s] * xv[s];
        y[r] = br + tt * -1.0;
    }
}

// stream floor: codes + b in, y out (MODE 1 bytes without the gathers)
__global__ __launch_bounds__(B) void kstream(const unsigned char *ell, const double *x, const double *b, double *y, int n)
{
    const int r = blockIdx.x * B + threadIdx.x;
    if (r >= n) return;
    const uint2 q = *reinterpret_cast<const uint2 *>(ell + (size_t)r * 8);
    y[r] = b[r] - x[r] * (double)(q.x ^ q.y);
}

// ---- engine replicas (sss_smooth.hip relax_range_ell MODE 0), for the ablation ------------------
struct XS {
    const double *f, *c;
    int split;
    __device__ __forceinline__ double operator()(int j) const { return j < split ? f[j] : c[j]; }
};
struct EllDict {
    int dd[32];
    double vd[8];
};
// BLK: row bounds from blk[]; PD: dictionaries through pd[]; XSEL: x through the two-pointer XSrc;
// RPT row blocks per workgroup
template <int RPT, bool BLK, bool PD, bool XSEL>
__global__ __launch_bounds__(B) void keng(const int2 *__restrict__ blk, const int4 *__restrict__ pd,
                                          const int *__restrict__ dd, const double *__restrict__ vd,
                                          const int *__restrict__ ddf, const double *__restrict__ vdf,
                                          const unsigned char *__restrict__ ell, const double *__restrict__ b, double *x,
                                          XS xs, int bend)
{
    __shared__ EllDict es[RPT];
    unsigned w[RPT][2];
    double br[RPT];
    int r[RPT];
    bool live[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int bid = blockIdx.x * RPT + j;
        live[j] = false;
        br[j] = 0.0;
        r[j] = 0;
        w[j][0] = w[j][1] = 0u;
        if (bid < bend) {
            int e;
            if (BLK) {
                const int2 ba = blk[bid], be = blk[bid + 1];
                r[j] = ba.x + (int)threadIdx.x;
                e = be.x;
            } else {
                r[j] = bid * B + (int)threadIdx.x;
                e = (bid + 1) * B;
            }
            live[j] = r[j] < e;
            if (live[j]) {
                const uint2 q = *reinterpret_cast<const uint2 *>(ell + (size_t)r[j] * 8);
                w[j][0] = q.x, w[j][1] = q.y;
                br[j] = b[r[j]];
            }
            if (PD) {
                const int4 p = pd[bid];
                if ((int)threadIdx.x < p.y) es[j].dd[threadIdx.x] = dd[p.x + threadIdx.x];
                if ((int)threadIdx.x < p.w) es[j].vd[threadIdx.x] = vd[p.z + threadIdx.x];
            } else {
                if (threadIdx.x < 32) es[j].dd[threadIdx.x] = ddf[(size_t)bid * 32 + threadIdx.x];
                else if (threadIdx.x < 40) es[j].vd[threadIdx.x - 32] = vdf[(size_t)bid * 8 + threadIdx.x - 32];
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        if (!live[j]) continue;
        const int rj = r[j];
        int c[8], len = 8, ds = -1;
        double a[8], p[8], dv = 0.0;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const unsigned byte = (w[j][s >> 2] >> (8 * (s & 3))) & 0xffu;
            if (byte == 0xffu && len == 8) len = s;
            c[s] = rj + es[j].dd[byte & 31u];
            a[s] = es[j].vd[byte >> 5];
        }
#pragma unroll
        for (int s = 0; s < 8; ++s)
            if (s < len && c[s] == rj) ds = s, dv = a[s];
#pragma unroll
        for (int s = 0; s < 8; ++s) p[s] = (s < len && s != ds) ? a[s] * (XSEL ? xs(c[s]) : x[c[s]]) : 0.0;
        double t = br[j];
#pragma unroll
        for (int s = 0; s < 8; ++s)
            if (s < len && s != ds) t -= p[s];
        if (fabs(dv) > 1e-20) x[rj] = t / dv;
    }
}

int main(int argc, char **argv)
{
    const int N = argc > 1 ? atoi(argv[1]) : 400;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const long long nn = (long long)N * N * N;
    const int n = (int)nn;
    // red-black relabel: F = odd (i+j+k), first; C = even, second; ascending original index in each
    std::vector<int> newid(n);
    int nF = 0;
    for (int g = 0; g < n; ++g) {
        const int i = g % N, j = (g / N) % N, k = g / (N * N);
        if ((i + j + k) & 1) newid[g] = nF++;
    }
    {
        int nc = nF;
        for (int g = 0; g < n; ++g) {
            const int i = g % N, j = (g / N) % N, k = g / (N * N);
            if (!((i + j + k) & 1)) newid[g] = nc++;
        }
    }
    if (nF % (4 * B) || (n - nF) % 4) { fprintf(stderr, "sizes not multiples of the blocking\n"); return 1; }
    std::vector<int> oldid(n);
    for (int g = 0; g < n; ++g) oldid[newid[g]] = g;
    const int nb = (n + B - 1) / B;
    std::vector<unsigned char> ell((size_t)n * 8, 0xff);
    std::vector<int> ddf((size_t)nb * 32, 0);
    std::vector<double> vdf((size_t)nb * 8, 0.0);
    int maxd = 0;
    for (int q = 0; q < nb; ++q) {
        int nd = 0;
        vdf[(size_t)q * 8] = -1.0, vdf[(size_t)q * 8 + 1] = 6.0;
        for (int r = q * B; r < std::min(n, (q + 1) * B); ++r) {
            const int g = oldid[r];
            const int i = g % N, j = (g / N) % N, k = g / (N * N);
            const int nbr[7] = {g - N * N, g - N, g - 1, g, g + 1, g + N, g + N * N};
            const bool in[7] = {k > 0, j > 0, i > 0, true, i < N - 1, j < N - 1, k < N - 1};
            int s = 0;
            for (int t = 0; t < 7; ++t) {
                if (!in[t]) continue;
                const int off = newid[nbr[t]] - r;
                int d = 0;
                while (d < nd && ddf[(size_t)q * 32 + d] != off) ++d;
                if (d == nd) {
                    if (nd == 31) { fprintf(stderr, "dictionary overflow\n"); return 1; }
                    ddf[(size_t)q * 32 + nd++] = off;
                }
                ell[(size_t)r * 8 + s++] = (unsigned char)((t == 3 ? 1 : 0) << 5 | d);
            }
        }
        maxd = std::max(maxd, nd);
    }
    printf("N=%d n=%d nF=%d max offsets per block %d\n", N, n, nF, maxd);
    unsigned char *d_ell;
    int *d_ddf;
    double *d_vdf, *x, *b, *y, *xs;
    CK(hipMalloc(&d_ell, ell.size()));
    CK(hipMalloc(&d_ddf, ddf.size() * 4));
    CK(hipMalloc(&d_vdf, vdf.size() * 8));
    CK(hipMalloc(&x, (size_t)n * 8));
    CK(hipMalloc(&xs, (size_t)n * 8));
    CK(hipMalloc(&b, (size_t)n * 8));
    CK(hipMalloc(&y, (size_t)n * 8));
    CK(hipMemcpy(d_ell, ell.data(), ell.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ddf, ddf.data(), ddf.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_vdf, vdf.data(), vdf.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> hx(n), hb(n);
    for (int r = 0; r < n; ++r) hx[r] = 1.0 + 1e-3 * (r % 977), hb[r] = 1.0 - 1e-3 * (r % 331);
    CK(hipMemcpy(xs, hx.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(b, hb.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> ref, got(n);
    auto run = [&](const char *name, int mode, double bytes, auto launch) {
        CK(hipMemcpy(x, xs, (size_t)n * 8, hipMemcpyDeviceToDevice));
        launch();   // the checked launch (an F pass from the same x each time)
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), (mode == 0 || mode == 2) ? x : y, (size_t)n * 8, hipMemcpyDeviceToHost));
        const char *chk = "";
        if (mode >= 0) {
            if (ref.empty() || mode >= 2) ref = got, chk = " (reference)";
            else {
                long long bad = 0, first = -1;
                for (int r = 0; r < n; ++r)
                    if (memcmp(&ref[r], &got[r], 8)) {
                        if (first < 0) first = r;
                        ++bad;
                    }
                chk = bad ? " MISMATCH" : " bitwise ok";
                if (bad) printf("   %lld rows differ, first %lld: %.17g vs %.17g\n", bad, first, ref[first], got[first]);
            }
        }
        for (int w = 0; w < 3; ++w) launch();
        CK(hipEventRecord(e0));
        for (int t = 0; t < reps; ++t) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-30s %8.1f us  %7.0f GB/s (%4.1f%% of 8 TB/s)%s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
               100.0 * bytes / (ms * 1e-3) / 8e12, chk);
        fflush(stdout);
    };
    // F pass bytes: codes + b + x_F written + x_C read once (the other class)
    const double fbytes = (double)nF * (8 + 8 + 8) + (double)(n - nF) * 8;
    const double rbytes = (double)n * (8 + 8 + 8 + 8);
#define FP(R, P) [&] { hipLaunchKernelGGL((kpass<0, R, P>), dim3(nF / (R * B)), dim3(B), 0, 0, d_ell, d_ddf, d_vdf, b, x, y, 0, nF); }
#define RS(R, P) [&] { hipLaunchKernelGGL((kpass<1, R, P>), dim3((n + R * B - 1) / (R * B)), dim3(B), 0, 0, d_ell, d_ddf, d_vdf, b, x, y, 0, n); }
    run("F pass R1", 2, fbytes, FP(1, false));
    run("F pass R2 scalar", 0, fbytes, FP(2, false));
    run("F pass R2 pair", 0, fbytes, FP(2, true));
    run("F pass R4 scalar", 0, fbytes, FP(4, false));
    run("F pass R4 pair", 0, fbytes, FP(4, true));
    {   // engine-shaped block bounds and dictionary descriptors
        std::vector<int2> blk(nb + 1);
        std::vector<int4> pd(nb);
        for (int q = 0; q < nb; ++q) blk[q] = make_int2(q * B, 0), pd[q] = make_int4(q * 32, 32, q * 8, 8);
        blk[nb] = make_int2(n, 0);
        int2 *d_blk;
        int4 *d_pd;
        CK(hipMalloc(&d_blk, blk.size() * 8));
        CK(hipMalloc(&d_pd, pd.size() * 16));
        CK(hipMemcpy(d_blk, blk.data(), blk.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_pd, pd.data(), pd.size() * 16, hipMemcpyHostToDevice));
        const XS xsel{x, x, 0x7fffffff};
        const int fb = nF / B;
#define EN(RPT, BL, PDV, XSV) [&] { hipLaunchKernelGGL((keng<RPT, BL, PDV, XSV>), dim3((fb + RPT - 1) / RPT), dim3(B), 0, 0, d_blk, d_pd, d_ddf, d_vdf, d_ddf, d_vdf, d_ell, b, x, xsel, fb); }
        run("eng rpt2 blk pd xsrc", 0, fbytes, EN(2, true, true, true));
        run("eng rpt1 blk pd xsrc", 0, fbytes, EN(1, true, true, true));
        run("eng rpt2 blk pd", 0, fbytes, EN(2, true, true, false));
        run("eng rpt2 pd xsrc", 0, fbytes, EN(2, false, true, true));
        run("eng rpt2 blk xsrc", 0, fbytes, EN(2, true, false, true));
        run("eng rpt2 (none)", 0, fbytes, EN(2, false, false, false));
        run("eng rpt1 (none)", 0, fbytes, EN(1, false, false, false));
    }
    for (int g : {512, 1024, 2048, 4096}) {
        char nm[64];
        snprintf(nm, sizeof nm, "F pass pipe G=%d", g);
        run(nm, 0, fbytes, [&] { hipLaunchKernelGGL(kpipe<0>, dim3(g), dim3(B), 0, 0, d_ell, d_ddf, d_vdf, b, x, y, 0, nF); });
    }
    run("resid R1", 3, rbytes, RS(1, false));
    for (int g : {512, 1024, 2048, 4096}) {
        char nm[64];
        snprintf(nm, sizeof nm, "resid pipe G=%d", g);
        run(nm, 1, rbytes, [&] { hipLaunchKernelGGL(kpipe<1>, dim3(g), dim3(B), 0, 0, d_ell, d_ddf, d_vdf, b, x, y, 0, n); });
    }
    run("resid R2 scalar", 1, rbytes, RS(2, false));
    run("resid R2 pair", 1, rbytes, RS(2, true));
    run("resid R4 scalar", 1, rbytes, RS(4, false));
    run("resid R4 pair", 1, rbytes, RS(4, true));
    {   // LDS-staged x: plans for the F pass (diagonal offset not staged) and the residual
        auto build = [&](bool with_diag, int lo_r, int hi_r) {
            std::vector<StagePlan> pl(nb);
            int staged = 0, maxr = 0, tot = 0;
            for (int q = 0; q < nb; ++q) {
                StagePlan &P = pl[q];
                memset(&P, 0, sizeof P);
                for (int d = 0; d < 32; ++d) P.lofs[d] = -1;
                const int r0 = q * B, r1 = std::min(n, r0 + B);
                if (r1 <= lo_r || r0 >= hi_r) { P.nr = -1; continue; }
                // offsets used by the block's rows
                bool used[32] = {};
                for (int r = r0; r < r1; ++r)
                    for (int sl = 0; sl < 8; ++sl) {
                        const unsigned char by = ell[(size_t)r * 8 + sl];
                        if (by == 0xff) break;
                        const int dgi = by & 31;
                        if (!with_diag && ddf[(size_t)q * 32 + dgi] == 0) continue;
                        used[dgi] = true;
                    }
                std::vector<std::pair<int, int>> iv;   // [start, end) global, per used offset
                std::vector<int> ofd;
                for (int dgi = 0; dgi < 32; ++dgi)
                    if (used[dgi]) {
                        const int o = ddf[(size_t)q * 32 + dgi];
                        iv.push_back({std::max(0, r0 + o), std::min(n, r1 + o)});
                        ofd.push_back(dgi);
                    }
                std::vector<int> ord(iv.size());
                for (size_t k = 0; k < ord.size(); ++k) ord[k] = (int)k;
                std::sort(ord.begin(), ord.end(), [&](int a2, int b2) { return iv[a2].first < iv[b2].first; });
                int nr = 0, lb = 0;
                bool ok = true;
                for (size_t k = 0; k < ord.size() && ok; ++k) {
                    const auto &I = iv[ord[k]];
                    if (nr > 0 && I.first <= P.gs[nr - 1] + P.len[nr - 1] + 16) {   // merge
                        const int e = std::max(P.gs[nr - 1] + P.len[nr - 1], I.second);
                        lb += e - (P.gs[nr - 1] + P.len[nr - 1]);
                        P.len[nr - 1] = e - P.gs[nr - 1];
                    } else {
                        if (nr == SR) { ok = false; break; }
                        P.gs[nr] = I.first, P.len[nr] = I.second - I.first, P.lb[nr] = lb;
                        lb += P.len[nr];
                        ++nr;
                    }
                }
                if (!ok || lb > SBUD) { P.nr = -1; continue; }
                for (size_t k = 0; k < iv.size(); ++k) {   // lofs: LDS index of row r0's value
                    const int o = ddf[(size_t)q * 32 + ofd[k]];
                    for (int m = 0; m < nr; ++m)
                        if (r0 + o >= P.gs[m] - B && r0 + o < P.gs[m] + P.len[m] &&
                            std::max(0, r0 + o) >= P.gs[m] && std::min(n, r1 + o) <= P.gs[m] + P.len[m]) {
                            P.lofs[ofd[k]] = P.lb[m] + (r0 + o - P.gs[m]);
                            break;
                        }
                }
                P.nr = nr;
                ++staged;
                maxr = std::max(maxr, nr);
                tot += lb;
            }
            printf("stage plan (%s): %d of %d blocks staged, max ranges %d, avg staged doubles %.0f\n",
                   with_diag ? "resid" : "F pass", staged, nb, maxr, staged ? (double)tot / staged : 0.0);
            StagePlan *dp;
            CK(hipMalloc(&dp, pl.size() * sizeof(StagePlan)));
            CK(hipMemcpy(dp, pl.data(), pl.size() * sizeof(StagePlan), hipMemcpyHostToDevice));
            return dp;
        };
        StagePlan *pf = build(false, 0, nF), *pr = build(true, 0, n);
        ref.clear();
        run("F pass R1 (again, reference)", 2, fbytes, FP(1, false));
        run("F pass staged", 0, fbytes, [&] { hipLaunchKernelGGL(kstage<0>, dim3(nF / B), dim3(B), 0, 0, d_ell, d_ddf, d_vdf, pf, b, x, y, 0, nF); });
        run("resid R1 (again, reference)", 3, rbytes, RS(1, false));
        run("resid staged", 1, rbytes, [&] { hipLaunchKernelGGL(kstage<1>, dim3(nb), dim3(B), 0, 0, d_ell, d_ddf, d_vdf, pr, b, x, y, 0, n); });
    }
    run("stream floor (codes,b,x,y)", -1, rbytes, [&] { hipLaunchKernelGGL(kstream, dim3(nb), dim3(B), 0, 0, d_ell, x, b, y, n); });
    return 0;
}
