// sss_spmv_dev.hpp — device building blocks shared by the SpMV-shaped kernels.
//
// csr_block_rows(): one workgroup = one CSR-adaptive row block (see sss_spmv.hip).  Each
// row's sum is formed from 0.0 in stored CSR order (the reference's order, SSS_utils.c:174 and
// Solve/SSS_cuda.cu:89-92), then handed to `epi(row, sum)`, which writes the result and
// returns this thread's contribution to an optional block reduction.
#pragma once

#include "sss_engine.hpp"

namespace sss {

// Block numbers are the dispatch order.  Measured and rejected: an XCD-contiguous
// renumbering of the grid (V-cycle 37.4 -> 39.8 ms at 400^3) and, for the ELL kernels, runs of G
// consecutive blocks per XCD (level 0 unchanged within noise, fabric bytes 3.5 -> 2.6 GB).
__device__ __forceinline__ int xcd_bid() { return blockIdx.x; }

struct SpmvSmem {
    alignas(16) double v[kTileEntries];    // products a_k * x_{c_k} of the tile (chain_pipe16 reads pairs)
    double red[kBlock / 64];
    double d[kBlock];          // sorted tiles: the raw diagonal value of each row of the block
};

// Dictionary tiles (DevCSR::dv_*): the block's dictionaries and each staged entry's row in LDS.
struct DictSmem {
    int dd[256];
    double vd[256];
    unsigned char rowof[kTileEntries];
};
struct DevDict {
    const unsigned *code = nullptr;
    const int4 *pd = nullptr;   // indexed by the block number the kernel sees
    const int *dd = nullptr;
    const double *vd = nullptr;
    // value-dictionary sorted tiles (code null): the sorted tiles' slots and cluster bases (pb
    // indexed as pd) with a value index per slot
    const unsigned *pk = nullptr;
    const unsigned char *vi = nullptr;
    const int2 *pb = nullptr;
    int tree_long = 0;   // DevCSR::tree_long (set for every matrix, dictionary or not)
    const unsigned char *ell = nullptr;   // dictionary ELL (DevCSR::dv_ell), ell_w bytes per row
    const int *ellb = nullptr;            // its per-row base columns (DevCSR::dv_ell_base) or null
    int ellw = 0;
    int bend = 0x7fffffff;   // ELL launches: first block past the launch's range (kEllRpt blocks per workgroup)
    const unsigned *xell = nullptr;   // column ELL (DevCSR::dv_xell), W 32-bit codes per row
    int xshift = 0;                   // its column bits (DevCSR::xell_shift)
};
// Dictionary ELL: row blocks per workgroup (each thread takes one row of each; more independent
// loads in flight per thread, one dictionary barrier for all of them).  Measured at 400^3
// (tools/gpu/ab.sh): 2 blocks took level 0's smoothing 3.12 -> 3.02 ms and its residual 389 ->
// 374 us per V-cycle; 4 blocks (70 VGPRs) were slower than 1 (3.36 ms).
constexpr int kEllRpt = 2;

// ---- dictionary ELL: one thread per row ----------------------------------------------------
// The block's dictionaries in LDS (small: the kernels instantiated for ELL keep their LDS
// footprint to this, so occupancy is not bounded by the tile staging arrays).
struct EllSmem {
    int dd[32];
    double vd[8];
    double red[kBlock / 64];
};
__device__ __forceinline__ void ell_load_dicts_nosync(const DevDict &dt, int bid, EllSmem &es)
{
    const int4 p = dt.pd[bid];
    if ((int)threadIdx.x < p.y) es.dd[threadIdx.x] = dt.dd[p.x + threadIdx.x];
    if ((int)threadIdx.x < p.w) es.vd[threadIdx.x] = dt.vd[p.z + threadIdx.x];
}
__device__ __forceinline__ void ell_load_dicts(const DevDict &dt, int bid, EllSmem &es)
{
    ell_load_dicts_nosync(dt, bid, es);
    __syncthreads();
}
// Row r's W code bytes (one 8/16/32-byte load).  The kernels issue it before the dictionaries'
// barrier: it depends only on the block bounds, so it overlaps the dictionary loads.
template <int W>
__device__ __forceinline__ void ell_codes(const unsigned char *__restrict__ ell, int r, unsigned (&w)[W / 4])
{
    if constexpr (W == 8) {
        const uint2 q = *reinterpret_cast<const uint2 *>(ell + (size_t)r * 8);
        w[0] = q.x, w[1] = q.y;
    } else {
#pragma unroll
        for (int h = 0; h < W / 16; ++h) {
            const uint4 q = *reinterpret_cast<const uint4 *>(ell + (size_t)r * W + 16 * h);
            w[4 * h] = q.x, w[4 * h + 1] = q.y, w[4 * h + 2] = q.z, w[4 * h + 3] = q.w;
        }
    }
}
// Products of row r in stored (slot) order from its codes: p[s] = a_s * x(c_s) for s < len;
// dslot = the row's (last) diagonal slot or -1, dval its value.  DIAG = false: the caller never
// reads p[dslot] (a relaxation pass subtracts every other product), so x_r is not fetched for it
// and p[dslot] = 0 -- the pass then reads no x of its own rows.
template <int W, bool DIAG = true, class Fetch>
__device__ __forceinline__ int ell_decode(const unsigned (&w)[W / 4], int r, const EllSmem &es, Fetch fetch,
                                          double (&p)[W], int &dslot, double &dval)
{
    int len = W;
    dslot = -1;
    dval = 0.0;
    int c[W];
    double a[W];
#pragma unroll
    for (int s = 0; s < W; ++s) {
        const unsigned byte = (w[s >> 2] >> (8 * (s & 3))) & 0xffu;
        if (byte == 0xffu && len == W) len = s;
        c[s] = r + es.dd[byte & 31u];
        a[s] = es.vd[byte >> 5];
    }
#pragma unroll
    for (int s = 0; s < W; ++s)
        if (s < len && c[s] == r) dslot = s, dval = a[s];
    // every gather issued before any product: with the multiply under the load's condition the
    // compiler waited for each load inside its branch (one HBM round trip per slot, in series)
    double xv[W];
#pragma unroll
    for (int s = 0; s < W; ++s) xv[s] = (s < len && (DIAG || s != dslot)) ? fetch(c[s]) : 0.0;
    // masked slots (past the row, the skipped diagonal) hold a * 0.0; no caller sums them
#pragma unroll
    for (int s = 0; s < W; ++s) p[s] = a[s] * xv[s];
    return len;
}
template <int W, class Fetch>
__device__ __forceinline__ int ell_row(const unsigned char *__restrict__ ell, int r, const EllSmem &es, Fetch fetch,
                                       double (&p)[W], int &dslot, double &dval)
{
    unsigned w[W / 4];
    ell_codes<W>(ell, r, w);
    return ell_decode<W>(w, r, es, fetch, p, dslot, dval);
}
// ---- dictionary ELL, two consecutive rows per thread (W = 8) --------------------------------------
// A workgroup covers its kEllRpt = 2 row blocks as one run of rows [ra, re) (the blocks are
// consecutive: the first ends where the second starts, at `mid`); thread t takes rows ra + 2t and
// ra + 2t + 1, so the codes of both rows come in one 16-byte load and b, x, y move as 16-byte pairs
// (loads and stores of 8-byte aligned pairs: gfx950 takes them unaligned).  Each row is decoded
// with its own block's dictionaries and summed exactly as ell_decode / ell_add do: bitwise the
// one-row-per-thread kernels.  tools/l0_lab.hip (7-pt 400^3, relabeled level 0): residual
// 589 -> 542 us, class pass 290 -> 284 us.  Used by the relaxation kernels; the residual SpMV keeps
// one row per thread (measured in the cycle at 400^3: the pairs took the relaxation passes 3.5-4.6 %
// faster but the F-row residual 5 % slower, 280 -> 294 us per V-cycle).
constexpr bool kEllPairs = kEllRpt == 2;
struct alignas(8) CodePair {
    unsigned x, y, z, w;
};
struct alignas(8) DoublePair {
    double a, b;
};
struct EllPairRows {
    int r = 0, mid = 0;             // first row of the pair; first row of the workgroup's second block
    int end = 0;                    // one past the workgroup's last row
    bool l0 = false, l1 = false;    // rows r, r + 1 exist
    bool v0 = false, v1 = false;    // the workgroup's blocks exist
    int b0 = 0;                     // the first block
};
__device__ __forceinline__ EllPairRows ell_pair_rows(const int2 *__restrict__ blk, int b0, int bend)
{
    EllPairRows p;
    p.b0 = b0;
    p.v0 = b0 < bend;
    p.v1 = b0 + 1 < bend;
    if (!p.v0) return p;
    const int ra = blk[b0].x;
    p.mid = blk[b0 + 1].x;
    const int re = p.v1 ? blk[b0 + 2].x : p.mid;
    p.end = re;
    p.r = ra + 2 * (int)threadIdx.x;
    p.l0 = p.r < re;
    p.l1 = p.r + 1 < re;
    return p;
}
// rows of the workgroup's two blocks together
__device__ __forceinline__ int ell_block_rows(const EllPairRows &p) { return p.end - (p.r - 2 * (int)threadIdx.x); }
// the pair's codes (rows r, r + 1), 0xFF... where a row does not exist
__device__ __forceinline__ void ell_pair_codes(const unsigned char *__restrict__ ell, const EllPairRows &p,
                                               unsigned (&w)[2][2])
{
    w[0][0] = w[0][1] = w[1][0] = w[1][1] = 0xffffffffu;
    if (p.l1) {
        const CodePair q = *reinterpret_cast<const CodePair *>(ell + (size_t)p.r * 8);
        w[0][0] = q.x, w[0][1] = q.y, w[1][0] = q.z, w[1][1] = q.w;
    } else if (p.l0) {
        const uint2 q = *reinterpret_cast<const uint2 *>(ell + (size_t)p.r * 8);
        w[0][0] = q.x, w[0][1] = q.y;
    }
}
__device__ __forceinline__ void pair_load(const double *__restrict__ v, int r, bool l0, bool l1, double (&o)[2])
{
    o[0] = o[1] = 0.0;
    if (l1) {
        const DoublePair q = *reinterpret_cast<const DoublePair *>(v + r);
        o[0] = q.a, o[1] = q.b;
    } else if (l0) {
        o[0] = v[r];
    }
}
__device__ __forceinline__ void pair_store(double *v, int r, bool l0, bool l1, const double (&o)[2])
{
    if (l1) {
        DoublePair q;
        q.a = o[0], q.b = o[1];
        *reinterpret_cast<DoublePair *>(v + r) = q;
    } else if (l0) {
        v[r] = o[0];
    }
}

// ---- column ELL: one thread per row, explicit columns ------------------------------------------
// Row r's W codes  value index << S | column  (0xFFFFFFFF pads) at xell[r * W], S = DevDict::xshift
// (the column bits of the matrix, >= 23), into the block's value dictionary (<= 2^(32 - S), at most
// 512 values) in LDS.
constexpr int kXellValues = 512;
struct XellSmem {
    double vd[kXellValues];
    double red[kBlock / 64];
};
__device__ __forceinline__ void xell_load_dict_nosync(const DevDict &dt, int bid, XellSmem &es)
{
    const int4 p = dt.pd[bid];
    for (int t = threadIdx.x; t < p.w; t += kBlock) es.vd[t] = dt.vd[p.z + t];
}
template <int W>
__device__ __forceinline__ void xell_codes(const unsigned *__restrict__ xell, int r, unsigned (&w)[W])
{
    static_assert(W % 4 == 0, "column ELL rows are whole 16-byte loads");
    const uint4 *q = reinterpret_cast<const uint4 *>(xell + (size_t)r * W);
#pragma unroll
    for (int h = 0; h < W / 4; ++h) {
        const uint4 u = q[h];
        w[4 * h] = u.x, w[4 * h + 1] = u.y, w[4 * h + 2] = u.z, w[4 * h + 3] = u.w;
    }
}
// Row r's x values in slot order, xv[s] = x(c_s) for s < len (0.0 past it); dslot = the row's
// (last) diagonal slot or -1 (DIAG = false: xv[dslot] = 0 without a fetch, as ell_decode).  The products a_s * xv[s] are formed where they are summed
// (xell_prod: the value from the LDS dictionary), so only the codes and the gathered x values
// stay in registers.
template <int W, bool DIAG = true, class Fetch>
__device__ __forceinline__ int xell_gather(const unsigned (&w)[W], int r, int shift, Fetch fetch, double (&xv)[W],
                                           int &dslot, unsigned &dcode)
{
    const unsigned mask = (1u << shift) - 1;
    int len = W;
    dslot = -1;
    dcode = 0u;
#pragma unroll
    for (int s = 0; s < W; ++s)
        if (w[s] == 0xffffffffu && len == W) len = s;
#pragma unroll
    for (int s = 0; s < W; ++s)
        if (s < len && (int)(w[s] & mask) == r) dslot = s, dcode = w[s];
#pragma unroll
    for (int s = 0; s < W; ++s) xv[s] = (s < len && (DIAG || s != dslot)) ? fetch((int)(w[s] & mask)) : 0.0;
    return len;
}
template <int W, bool DIAG = true, class Fetch>
__device__ __forceinline__ int xell_gather(const unsigned (&w)[W], int r, int shift, Fetch fetch, double (&xv)[W],
                                           int &dslot)
{
    unsigned dcode;
    return xell_gather<W, DIAG>(w, r, shift, fetch, xv, dslot, dcode);
}
// s0 + (or -) the products a_s * xv[s] of slots [a, e) in slot order, a_s = the block's value of slot
// s (LDS).  Branch-free form: every slot's LDS value is read first (slots outside [a, e) read entry 0)
// and each step is a select.  It holds W more doubles live than the per-slot form (xell_add /
// xell_sub): measured at 400^3 the two-stage stage-0 kernel ran 4 % faster with it, the level-1
// relaxation (122 VGPRs instead of 70: 4 waves per SIMD instead of 7) 3 % slower, so only the former uses it.
template <bool SUB, int W>
__device__ __forceinline__ double xell_sum_bf(double s0, const unsigned (&w)[W], const double (&xv)[W], const XellSmem &es,
                                              int shift, int a, int e)
{
    double av[W];
#pragma unroll
    for (int s = 0; s < W; ++s) av[s] = es.vd[(s >= a && s < e) ? (w[s] >> shift) : 0u];
#pragma unroll
    for (int s = 0; s < W; ++s) {
        const double p = av[s] * xv[s];
        const double t = SUB ? s0 - p : s0 + p;
        s0 = (s >= a && s < e) ? t : s0;
    }
    return s0;
}
// Per-slot form: a branch per slot, its LDS value read inside it (groups of values read ahead and
// selected per slot were measured no faster on level 1 at 400^3).
template <bool SUB, int W>
__device__ __forceinline__ double xell_sum_g(double s0, const unsigned (&w)[W], const double (&xv)[W], const XellSmem &es,
                                             int shift, int a, int e)
{
#pragma unroll
    for (int s = 0; s < W; ++s)
        if (s >= a && s < e) s0 = SUB ? s0 - es.vd[w[s] >> shift] * xv[s] : s0 + es.vd[w[s] >> shift] * xv[s];
    return s0;
}
template <int W>
__device__ __forceinline__ double xell_add(double s0, const unsigned (&w)[W], const double (&xv)[W], const XellSmem &es,
                                           int shift, int a, int e)
{
    return xell_sum_g<false>(s0, w, xv, es, shift, a, e);
}
template <int W>
__device__ __forceinline__ double xell_sub(double s0, const unsigned (&w)[W], const double (&xv)[W], const XellSmem &es,
                                           int shift, int a, int e)
{
    return xell_sum_g<true>(s0, w, xv, es, shift, a, e);
}

// sum of p[a, e) from s0 in slot order (branch-free: a select per slot)
template <int W>
__device__ __forceinline__ double ell_add(double s0, const double (&p)[W], int a, int e)
{
#pragma unroll
    for (int s = 0; s < W; ++s) {
        const double t = s0 + p[s];
        s0 = (s >= a && s < e) ? t : s0;
    }
    return s0;
}
template <int W>
__device__ __forceinline__ double ell_sub(double s0, const double (&p)[W], int a, int e)
{
#pragma unroll
    for (int s = 0; s < W; ++s) {
        const double t = s0 - p[s];
        s0 = (s >= a && s < e) ? t : s0;
    }
    return s0;
}

// In-order chains over LDS products: 8 reads issued ahead of 8 dependent adds/subtractions,
// the additions themselves in exactly the stored order.
__device__ __forceinline__ double chain_add(double s, const double *p, int a, int e)
{
    int k = a;
    for (; k + 8 <= e; k += 8) {
        const double p0 = p[k], p1 = p[k + 1], p2 = p[k + 2], p3 = p[k + 3];
        const double p4 = p[k + 4], p5 = p[k + 5], p6 = p[k + 6], p7 = p[k + 7];
        s += p0; s += p1; s += p2; s += p3; s += p4; s += p5; s += p6; s += p7;
    }
    for (; k < e; ++k) s += p[k];
    return s;
}
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

// The in-order chain with its schedule fixed: groups of G products read as 16-byte pairs into two
// register sets in turn, each group's G dependent adds in one asm block, so the compiler neither
// copies between the sets nor sinks the next group's reads below the current adds.  Written in plain
// C++ (16 reads ahead, then the adds, then a copy of the sets) inside a loop that also keeps global
// loads in flight, it did both: tools/row_chain_lab.hip on MI355X, one wave, a 2,907-entry row in
// 256-entry strips, 21.3 cycles per entry that way, 13.8 with this at G = 16; the bare chain over
// LDS 10.7 against 8.9, the dependent v_add_f64 floor 8.1 (tools/chain_lab.hip).  s + p[0] + ... + p[m-1] (SUB: s - ...), same bits.
// p 16-byte aligned in LDS; reads up to G entries past m (values unused), which must stay inside
// the LDS allocation.
#define SSS_ADD2(i, j) "v_add_f64 %0, %0, %" #i "\n\tv_add_f64 %0, %0, %" #j "\n\t"
#define SSS_SUB2(i, j) "v_add_f64 %0, %0, -%" #i "\n\tv_add_f64 %0, %0, -%" #j "\n\t"
#define SSS_OPS8(c) "v"(c[0].x), "v"(c[0].y), "v"(c[1].x), "v"(c[1].y), "v"(c[2].x), "v"(c[2].y), "v"(c[3].x), "v"(c[3].y)
#define SSS_OPS16(c)                                                                                            \
    SSS_OPS8(c), "v"(c[4].x), "v"(c[4].y), "v"(c[5].x), "v"(c[5].y), "v"(c[6].x), "v"(c[6].y), "v"(c[7].x), \
        "v"(c[7].y)
template <bool SUB, int G>
__device__ __forceinline__ double chain_group(double s, const double2 (&c)[G / 2])
{
    static_assert(G == 8 || G == 16, "group of 8 or 16");
    if constexpr (G == 8 && !SUB)
        asm volatile(SSS_ADD2(1, 2) SSS_ADD2(3, 4) SSS_ADD2(5, 6) SSS_ADD2(7, 8) : "+v"(s) : SSS_OPS8(c));
    else if constexpr (G == 8)
        asm volatile(SSS_SUB2(1, 2) SSS_SUB2(3, 4) SSS_SUB2(5, 6) SSS_SUB2(7, 8) : "+v"(s) : SSS_OPS8(c));
    else if constexpr (!SUB)
        asm volatile(SSS_ADD2(1, 2) SSS_ADD2(3, 4) SSS_ADD2(5, 6) SSS_ADD2(7, 8) SSS_ADD2(9, 10) SSS_ADD2(11, 12)
                         SSS_ADD2(13, 14) SSS_ADD2(15, 16)
                     : "+v"(s)
                     : SSS_OPS16(c));
    else
        asm volatile(SSS_SUB2(1, 2) SSS_SUB2(3, 4) SSS_SUB2(5, 6) SSS_SUB2(7, 8) SSS_SUB2(9, 10) SSS_SUB2(11, 12)
                         SSS_SUB2(13, 14) SSS_SUB2(15, 16)
                     : "+v"(s)
                     : SSS_OPS16(c));
    return s;
}
template <bool SUB, int G>
__device__ __forceinline__ double chain_fixed(double s, const double *p, int m)
{
    int k = 0;
    if (m >= 2 * G) {
        double2 a[G / 2], b[G / 2];
#pragma unroll
        for (int u = 0; u < G / 2; ++u) a[u] = *reinterpret_cast<const double2 *>(p + 2 * u);
        for (; k + 2 * G <= m; k += 2 * G) {
#pragma unroll
            for (int u = 0; u < G / 2; ++u) b[u] = *reinterpret_cast<const double2 *>(p + k + G + 2 * u);
            s = chain_group<SUB, G>(s, a);
#pragma unroll
            for (int u = 0; u < G / 2; ++u) a[u] = *reinterpret_cast<const double2 *>(p + k + 2 * G + 2 * u);
            s = chain_group<SUB, G>(s, b);
        }
        if (k + G <= m) {
            s = chain_group<SUB, G>(s, a);
            k += G;
        }
    }
    // the tail (and rows under 2 G): groups of 8 read together, then added
    for (; k + 8 <= m; k += 8) {
        double2 c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = *reinterpret_cast<const double2 *>(p + k + 2 * u);
        s = chain_group<SUB, 8>(s, c);
    }
    for (; k < m; ++k) s = SUB ? s - p[k] : s + p[k];
    return s;
}
#undef SSS_ADD2
#undef SSS_SUB2
#undef SSS_OPS8
#undef SSS_OPS16

// One lane's in-order chain over a long run of LDS products (the exact GS-CF engines, the parity
// wave-per-row kernels, the stored-order block rows): s -/+= p[a], p[a+1], ... in order -- chain_fixed
// after one entry that aligns the pair reads (p 16-byte aligned).  Reads up to 16 products past e
// (values unused): every caller's buffer continues in LDS or ends the allocation.
constexpr int kPipeRowMin = 64;   // csr_block_rows: rows from this length chain with chain_pipe16
template <bool SUB>
__device__ __forceinline__ double chain_pipe16(double s, const double *p, int a, int e)
{
    if ((a & 1) && a < e) s = SUB ? s - p[a++] : s + p[a++];
    return a < e ? chain_fixed<SUB, 16>(s, p + a, e - a) : s;
}

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

// Tree sum of the LDS products p[a, e) (thread-strided partial sums, block_sum): the free
// summation order of a long row's chunk (DevCSR::tree_long).  Result valid in thread 0; every
// thread of the block must call it.
__device__ __forceinline__ double block_tree_sum(const double *p, int a, int e, double *red)
{
    double t = 0.0;
    for (int k = a + (int)threadIdx.x; k < e; k += kBlock) t += p[k];
    return block_sum(t, red);
}

// Phase 1 of every tile kernel: sm[k - k0] = v[k] * x[ci[k]] for k in [k0, k1).  Each thread
// issues all its column/value loads of a batch first, then all its x gathers, so up to 8 + 8
// independent loads per thread are in flight (2x the bandwidth of the load-multiply loop on a
// 7-point operator).  A negative column (diagonal sentinel of the relaxation copies) stores an
// exact +0.0.
__device__ __forceinline__ void stage_products(double *__restrict__ sm, int k0, int k1, const int *__restrict__ ci,
                                               const double *__restrict__ v, const double *x)
{
    constexpr int U = 8;
    for (int kb = k0 + (int)threadIdx.x; kb < k1; kb += U * kBlock) {
        int j[U];
        double a[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb + u * kBlock;
            j[u] = k < k1 ? ci[k] : -1;
            a[u] = k < k1 ? v[k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = j[u] >= 0 ? x[j[u]] : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb + u * kBlock;
            if (k < k1) sm[k - k0] = j[u] >= 0 ? a[u] * xv[u] : 0.0;
        }
    }
}

// As stage_products, by `nt` threads of the block (this one is thread `t` of them).
__device__ __forceinline__ void stage_products_part(double *__restrict__ sm, int k0, int k1,
                                                    const int *__restrict__ ci, const double *__restrict__ v,
                                                    const double *x, int t, int nt)
{
    constexpr int U = 8;
    for (int kb = k0 + t; kb < k1; kb += U * nt) {
        int j[U];
        double a[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb + u * nt;
            j[u] = k < k1 ? ci[k] : -1;
            a[u] = k < k1 ? v[k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = j[u] >= 0 ? x[j[u]] : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb + u * nt;
            if (k < k1) sm[k - k0] = j[u] >= 0 ? a[u] * xv[u] : 0.0;
        }
    }
}

// As stage_products, with the x value of each (possibly encoded) column supplied by `fetch`.
template <class Fetch>
__device__ __forceinline__ void stage_products_f(double *__restrict__ sm, int k0, int k1, const int *__restrict__ ci,
                                                 const double *__restrict__ v, Fetch fetch)
{
    constexpr int U = 8;
    for (int kb = k0 + (int)threadIdx.x; kb < k1; kb += U * kBlock) {
        int c[U];
        double a[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb + u * kBlock;
            c[u] = k < k1 ? ci[k] : 0;
            a[u] = k < k1 ? v[k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = kb + u * kBlock < k1 ? fetch(c[u]) : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb + u * kBlock;
            if (k < k1) sm[k - k0] = a[u] * xv[u];
        }
    }
}

// Column-sorted staging (DevCSR::pk/pv/pb): slot k of the segment [k0, k1) holds the entry packed
// as cluster << 31 | (col - base[cluster]) << kTileShift | pos, pos = its stored-order position in
// the segment (a diagonal entry: offset kTileDiagMark + its row in the block); the product goes to
// sm[pos], so the LDS image is exactly stage_products_f's and every chain over it is unchanged.
template <class Fetch>
__device__ __forceinline__ void stage_sorted(double *__restrict__ sm, int k0, int k1, const unsigned *__restrict__ pk,
                                             const double *__restrict__ pv, int2 base, int r0, double *diag,
                                             Fetch fetch)
{
    constexpr int U = 8;
    constexpr unsigned kMask = kTileEntries - 1;
    for (int kb = k0 + (int)threadIdx.x; kb < k1; kb += U * kBlock) {
        unsigned q[U];
        double a[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb + u * kBlock;
            q[u] = k < k1 ? pk[k] : 0u;
            a[u] = k < k1 ? pv[k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned off = (q[u] >> kTileShift) & ((1u << kTileColBits) - 1);
            const int c = off >= kTileDiagMark ? r0 + (int)(off - kTileDiagMark) : (int)off + ((q[u] >> 31) ? base.y : base.x);
            xv[u] = kb + u * kBlock < k1 ? fetch(c) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (kb + u * kBlock < k1) {
                sm[q[u] & kMask] = a[u] * xv[u];
                const unsigned off = (q[u] >> kTileShift) & ((1u << kTileColBits) - 1);
                if (diag && off >= kTileDiagMark) diag[off - kTileDiagMark] = a[u];
            }
    }
}

// Value-dictionary sorted tiles: stage_sorted with the value of slot k read from the block's
// dictionary in LDS (vd[vi[k]], the same bit pattern pv[k] held).
// The slots of one pass of the loop below (U per thread): stage_dict loads the first pass ahead of
// the dictionary barrier, so the slot stream is in flight while the dictionary arrives.
constexpr int kVdictU = 8;
__device__ __forceinline__ void vdict_load(int kb, int k1, const unsigned *__restrict__ pk,
                                           const unsigned char *__restrict__ vi, unsigned (&q)[kVdictU],
                                           unsigned (&w)[kVdictU])
{
#pragma unroll
    for (int u = 0; u < kVdictU; ++u) {
        const int k = kb + u * kBlock;
        q[u] = k < k1 ? pk[k] : 0u;
        w[u] = k < k1 ? vi[k] : 0u;
    }
}
template <class Fetch>
__device__ __forceinline__ void stage_vdict(double *__restrict__ sm, int k0, int k1, const unsigned *__restrict__ pk,
                                            const unsigned char *__restrict__ vi, const double *vd, int2 base, int r0,
                                            double *diag, Fetch fetch, const unsigned (*pre_q)[kVdictU] = nullptr,
                                            const unsigned (*pre_w)[kVdictU] = nullptr)
{
    constexpr int U = kVdictU;
    constexpr unsigned kMask = kTileEntries - 1;
    for (int kb = k0 + (int)threadIdx.x; kb < k1; kb += U * kBlock) {
        unsigned q[U], w[U];
        double a[U], xv[U];
        if (pre_q && kb == k0 + (int)threadIdx.x) {
#pragma unroll
            for (int u = 0; u < U; ++u) q[u] = (*pre_q)[u], w[u] = (*pre_w)[u];
        } else {
            vdict_load(kb, k1, pk, vi, q, w);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned off = (q[u] >> kTileShift) & ((1u << kTileColBits) - 1);
            const int c = off >= kTileDiagMark ? r0 + (int)(off - kTileDiagMark) : (int)off + ((q[u] >> 31) ? base.y : base.x);
            xv[u] = kb + u * kBlock < k1 ? fetch(c) : 0.0;
            a[u] = vd[w[u]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (kb + u * kBlock < k1) {
                sm[q[u] & kMask] = a[u] * xv[u];
                const unsigned off = (q[u] >> kTileShift) & ((1u << kTileColBits) - 1);
                if (diag && off >= kTileDiagMark) diag[off - kTileDiagMark] = a[u];
            }
    }
}

// Dictionary tiles: slot k of segment [k0, k1) of block `bid` (rows [r0, r1)) holds
// code = value index << 19 | offset index << 11 | pos, pos = the entry's stored-order position in
// the segment (slots are in column order); col = row(pos) + dd[offset index], a = vd[value index];
// the product lands at sm[pos], so the LDS image is stage_products_f's.  Starts with a workgroup
// barrier of its own (the block's dictionaries and the position -> row map go to LDS first).
// PRE: issue the first pass of value-dictionary slot loads before the dictionary barrier (the
// relaxation kernels gain from it; measured slower in the SpMV kernels, which keep the plain order)
template <bool PRE = true, class Fetch>
__device__ __forceinline__ void stage_dict(double *__restrict__ sm, int k0, int k1, const DevDict &dt, int bid,
                                           int r0, int r1, const int *__restrict__ rp, DictSmem &ds, double *diag,
                                           Fetch fetch)
{
    const int4 p = dt.pd[bid];
    if (dt.vi) {   // value-dictionary sorted tiles: stage_sorted with a[k] = vd[vi[k]]
        if constexpr (PRE) {
            unsigned q[kVdictU], w[kVdictU];
            vdict_load(k0 + (int)threadIdx.x, k1, dt.pk, dt.vi, q, w);   // in flight across the barrier
            const int2 base = dt.pb[bid];
            for (int t = threadIdx.x; t < p.w; t += kBlock) ds.vd[t] = dt.vd[p.z + t];
            __syncthreads();
            stage_vdict(sm, k0, k1, dt.pk, dt.vi, ds.vd, base, r0, diag, fetch, &q, &w);
        } else {
            for (int t = threadIdx.x; t < p.w; t += kBlock) ds.vd[t] = dt.vd[p.z + t];
            __syncthreads();
            stage_vdict(sm, k0, k1, dt.pk, dt.vi, ds.vd, dt.pb[bid], r0, diag, fetch);
        }
        return;
    }
    for (int t = threadIdx.x; t < p.w; t += kBlock) ds.vd[t] = dt.vd[p.z + t];
    for (int t = threadIdx.x; t < p.y; t += kBlock) ds.dd[t] = dt.dd[p.x + t];
    for (int r = r0 + (int)threadIdx.x; r < r1; r += kBlock) {
        const int a = max(rp[r], k0), e = min(rp[r + 1], k1);
        for (int k = a; k < e; ++k) ds.rowof[k - k0] = (unsigned char)(r - r0);
    }
    __syncthreads();
    constexpr int U = 8;
    constexpr unsigned kMask = kTileEntries - 1;
    for (int kb = k0 + (int)threadIdx.x; kb < k1; kb += U * kBlock) {
        unsigned q[U];
        int c[U], rw[U];
        double a[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb + u * kBlock;
            q[u] = k < k1 ? dt.code[k] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            rw[u] = ds.rowof[q[u] & kMask];
            c[u] = r0 + rw[u] + ds.dd[(q[u] >> kTileShift) & 255u];
            a[u] = ds.vd[(q[u] >> (kTileShift + 8)) & 255u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = kb + u * kBlock < k1 ? fetch(c[u]) : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (kb + u * kBlock < k1) {
                sm[q[u] & kMask] = a[u] * xv[u];
                if (diag && c[u] == r0 + rw[u]) diag[rw[u]] = a[u];
            }
    }
}

// Stage the products of segment [k0, k1) of block `bid` (first row r0): from the sorted copy when
// the matrix has one (then diag[row - r0], if given, receives each row's diagonal value).
template <class Fetch>
__device__ __forceinline__ void stage_any(double *__restrict__ sm, int k0, int k1, const int *__restrict__ ci,
                                          const double *__restrict__ v, const unsigned *__restrict__ pk,
                                          const double *__restrict__ pv, const int2 *__restrict__ pb, int bid, int r0,
                                          double *diag, Fetch fetch)
{
    if (pk) stage_sorted(sm, k0, k1, pk, pv, pb[bid], r0, diag, fetch);
    else stage_products_f(sm, k0, k1, ci, v, fetch);
}
// ... or from the dictionary tiles when ds is given (kernels instantiated for them)
template <class Fetch>
__device__ __forceinline__ void stage_any(double *__restrict__ sm, int k0, int k1, const int *__restrict__ ci,
                                          const double *__restrict__ v, const unsigned *__restrict__ pk,
                                          const double *__restrict__ pv, const int2 *__restrict__ pb, int bid, int r0,
                                          double *diag, Fetch fetch, const DevDict &dt, DictSmem *ds, int r1,
                                          const int *__restrict__ rp)
{
    if (ds) stage_dict(sm, k0, k1, dt, bid, r0, r1, rp, *ds, diag, fetch);
    else stage_any(sm, k0, k1, ci, v, pk, pv, pb, bid, r0, diag, fetch);
}

// Returns this thread's summed epilogue contribution (0 for idle threads).
// Phase 1: every thread of the workgroup forms products of the tile (coalesced val/col loads,
// independent x gathers, all in flight).  Phase 2: one thread per row adds its products from
// LDS in stored order starting from 0.0 (SSS_utils.c:174).  Rows longer than the tile are
// processed alone, tile by tile, with thread 0 carrying the chain.
// A block's row and entry bounds: from {row, entry} pairs (one load each side) or from the
// first-row array through row_ptr.
struct BlockBounds {
    int r0, r1, k0, k1;
};
__device__ __forceinline__ BlockBounds block_bounds(const int2 *__restrict__ bk, const int *__restrict__, int bid)
{
    const int2 a = bk[bid], e = bk[bid + 1];
    return {a.x, e.x, a.y, e.y};
}
__device__ __forceinline__ BlockBounds block_bounds(const int *__restrict__ blk, const int *__restrict__ rp, int bid)
{
    const int r0 = blk[bid], r1 = blk[bid + 1];
    return {r0, r1, rp[r0], rp[r1]};
}

template <class Epi, class BlkT>
__device__ __forceinline__ double csr_block_rows(const BlkT *__restrict__ blk, const int *__restrict__ rp,
                                                 const int *__restrict__ ci, const double *__restrict__ v,
                                                 const double *__restrict__ x, SpmvSmem &sm, Epi epi,
                                                 const unsigned *__restrict__ pk = nullptr,
                                                 const double *__restrict__ pv = nullptr,
                                                 const int2 *__restrict__ pb = nullptr, const DevDict *dt = nullptr,
                                                 DictSmem *ds = nullptr)
{
    auto fetch = [&](int c) -> double { return x[c]; };
    const int bid = xcd_bid();
    const BlockBounds bb = block_bounds(blk, rp, bid);
    const int r0 = bb.r0, r1 = bb.r1, k0 = bb.k0, k1 = bb.k1;
    const int cnt = k1 - k0;
    double contrib = 0.0;
    if (cnt <= kTileEntries) {
        const int r = r0 + (int)threadIdx.x;
        int ra = 0, re = 0;
        if (r < r1) ra = rp[r], re = rp[r + 1];   // issued ahead of the tile
        if (ds) stage_dict<false>(sm.v, k0, k1, *dt, bid, r0, r1, rp, *ds, (double *)nullptr, fetch);
        else if (pk) stage_sorted(sm.v, k0, k1, pk, pv, pb[bid], r0, (double *)nullptr, fetch);
        else stage_products(sm.v, k0, k1, ci, v, x);
        __syncthreads();
        if (r < r1) {
            // rows of 64+ entries: the pipelined chain (same additions in the same order)
            const double s = re - ra >= kPipeRowMin ? chain_pipe16<false>(0.0, sm.v, ra - k0, re - k0)
                                                    : chain_add(0.0, sm.v, ra - k0, re - k0);
            contrib = epi(r, s);
        }
    } else if (!ds && !pk) {
        // one long row, plain CSR: halves of the tile as a double buffer -- wave 0's lane 0 chains
        // one half while waves 1-3 stage the next (the same additions in the same order)
        constexpr int H = kTileEntries / 2;
        double s = 0.0;
        stage_products(sm.v, k0, min(k0 + H, k1), ci, v, x);
        __syncthreads();
        for (int base = k0, c = 0; base < k1; base += H, ++c) {
            const int m = min(H, k1 - base), nb = base + H;
            double *cur = sm.v + (c & 1) * H, *nxt = sm.v + ((c + 1) & 1) * H;
            if (threadIdx.x == 0) s = chain_pipe16<false>(s, cur, 0, m);
            else if (threadIdx.x >= 64 && nb < k1)
                stage_products_part(nxt, nb, min(nb + H, k1), ci, v, x, (int)threadIdx.x - 64, kBlock - 64);
            __syncthreads();
        }
        if (threadIdx.x == 0) contrib = epi(r0, s);
    } else {
        double s = 0.0;
        for (int base = k0; base < k1; base += kTileEntries) {
            const int m = min(kTileEntries, k1 - base);
            if (ds) stage_dict<false>(sm.v, base, base + m, *dt, bid, r0, r1, rp, *ds, (double *)nullptr, fetch);
            else if (pk) stage_sorted(sm.v, base, base + m, pk, pv, pb[bid], r0, (double *)nullptr, fetch);
            else stage_products(sm.v, base, base + m, ci, v, x);
            __syncthreads();
            if (dt && dt->tree_long) {
                const double c = block_tree_sum(sm.v, 0, m, sm.red);
                if (threadIdx.x == 0) s += c;
            } else if (threadIdx.x == 0) {
                s = chain_pipe16<false>(s, sm.v, 0, m);
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) contrib = epi(r0, s);
    }
    return contrib;
}



}  // namespace sss

namespace sss {

// Relaxation rows over a row-compacted CSR (one smoother class): local row r is global row
// map[r]; diagonal entries carry column -1 (set at upload) so their product is +0.0, an exact
// identity for subtraction.  The chain is  acc = b_i;  acc -= a_k * x_{j_k}  for every
// off-diagonal entry in stored order — exactly Solve/SSS_smooth.c:21-26 — then `epi(r, i, acc)`.
template <class Epi>
__device__ __forceinline__ void csr_block_relax(const int *__restrict__ blk, const int *__restrict__ rp,
                                                const int *__restrict__ ci, const double *__restrict__ v,
                                                const int *__restrict__ map, const double *__restrict__ b,
                                                const double *x, SpmvSmem &sm, Epi epi)
{
    const int bid = xcd_bid();
    const int r0 = blk[bid], r1 = blk[bid + 1];
    const int k0 = rp[r0], k1 = rp[r1];
    const int cnt = k1 - k0;
    if (cnt <= kTileEntries) {
        const int r = r0 + (int)threadIdx.x;
        int ra = 0, re = 0, i = 0;
        if (r < r1) ra = rp[r], re = rp[r + 1], i = map[r];
        stage_products(sm.v, k0, k1, ci, v, x);
        __syncthreads();
        if (r < r1) {
            const double acc = chain_sub(b[i], sm.v, ra - k0, re - k0);
            epi(r, i, acc);
        }
    } else {
        const int i = map[r0];
        double acc = b[i];
        for (int base = k0; base < k1; base += kTileEntries) {
            const int m = min(kTileEntries, k1 - base);
            stage_products(sm.v, base, base + m, ci, v, x);
            __syncthreads();
            if (threadIdx.x == 0) acc = chain_sub(acc, sm.v, 0, m);
            __syncthreads();
        }
        if (threadIdx.x == 0) epi(r0, i, acc);
    }
}



}  // namespace sss

namespace sss {

// ---- wave-per-row path for long rows (avg nnz/row >= kWaveRowMin) ----------------------------
// Four rows per 256-thread workgroup, one per wave.  All 64 lanes gather a strip of the row's
// products (kWaveStage / 64 independent loads per lane) into the wave's private LDS strip; lane 0
// then runs the in-order chain over the strip.  LDS traffic of one wave is in order, so a
// wave-level fence is the only synchronisation needed.  Measured on the 7-pt 256^3 hierarchy
// (tools/lab_rows.py): the tile path wins up to ~400 entries per row, this path from ~700.
constexpr int kWaveStage = 256;    // doubles per wave strip (2 KiB; 8 KiB per workgroup)
constexpr int kWaveRowMin = 600;   // average entries per row from which a matrix uses this path
// Free order (throughput mode): average entries per row from which a matrix is summed in tree
// order -- merged row groups beat the bitwise sorted tiles from ~300 (7-pt 400^3 level 5: 183 vs
// 243 us per residual, level 4 at 199 per row: 145 vs 133 us, tools/lab_rows.hip).
constexpr int kFreeRowMin = 300;

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// SUB = false: returns init + p_0 + p_1 + ...;  SUB = true: init - p_0 - p_1 - ...  (stored order)
// with p_k = prod(col_k, val_k).  Result valid in lane 0 of the wave.
template <bool SUB, class Prod>
__device__ __forceinline__ double wave_row_chain(int k0, int k1, const int *__restrict__ ci,
                                                 const double *__restrict__ v, Prod prod, double init,
                                                 double *strip)
{
    constexpr int U = kWaveStage / 64;
    const int lane = threadIdx.x & 63;
    double acc = init;
    for (int base = k0; base < k1; base += kWaveStage) {
        const int m = min(kWaveStage, k1 - base);
        int c[U];
        double a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {   // unconditional loads (clamped into the row): no branch per load
            const int q = lane + 64 * u, qc = q < m ? q : m - 1;
            const int cv = ci[base + qc];
            const double av = v[base + qc];
            c[u] = cv;
            a[u] = q < m ? av : 0.0;
        }
        // every product formed before any is stored (a lane past the row reuses the row's last column
        // with value 0.0, so an offset fetch stays inside its segment): with the store's condition
        // around it the compiler waited for each gather in turn
        double pv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) pv[u] = prod(c[u], a[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = lane + 64 * u;
            if (q < m) strip[q] = pv[u];
        }
        wave_sync();
        if (lane == 0) acc = chain_pipe16<SUB>(acc, strip, 0, m);
        wave_sync();
    }
    return acc;
}

// Free sum order (DevCSR::vec_rows): sum_k prod(col_k, val_k) over [k0, k1) by the whole wave --
// lane l takes entries k0 + l + 64 t (two interleaved accumulators, four loads in flight), then an
// xor-butterfly.  Fixed order, so deterministic; valid in every lane.
template <class Prod>
__device__ __forceinline__ double wave_row_sum(int k0, int k1, const int *__restrict__ ci,
                                               const double *__restrict__ v, Prod prod)
{
    constexpr int U = 4;
    const int lane = threadIdx.x & 63;
    double s0 = 0.0, s1 = 0.0;
    for (int k = k0 + lane; k < k1; k += 64 * U) {
        int c[U];
        double a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {   // unconditional loads (clamped into the row): no branch per load
            const int kk = k + 64 * u, kc = kk < k1 ? kk : k1 - 1;
            const int cv = ci[kc];
            const double av = v[kc];
            c[u] = cv;
            a[u] = kk < k1 ? av : 0.0;
        }
        // every gather issued before any is used (masked lanes: the row's last column, value 0.0, so
        // an offset fetch stays inside its segment; the product is dropped)
        double pv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) pv[u] = prod(c[u], a[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double p = k + 64 * u < k1 ? pv[u] : 0.0;
            if (u & 1) s1 += p;
            else s0 += p;
        }
    }
    double s = s0 + s1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}


// Merged row groups (DevCSR::mg_*): the entries [k0, k1) of one group, lane-strided with U loads in
// flight; lane l accumulates its entries in increasing position into the accumulator of the
// entry's (segment, row), then each accumulator's 64 lane sums are xor-reduced.  Fixed order:
// deterministic.  s0[u] / s1[u] = sum over row u's first- / second-segment entries of
// val * fetch(col), valid in every lane (S = 1: single-segment matrices, s1 untouched).

// (U, the loads in flight per lane, changes no sum: each lane still adds its entries in increasing
// position into the same accumulators)
template <int G, int S, class Fetch>
__device__ __forceinline__ void merged_sums(int k0, int k1, const unsigned *__restrict__ mk,
                                            const double *__restrict__ mv, Fetch fetch, double (&s0)[G],
                                            double (&s1)[G])
{
    constexpr int U = 8;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < G; ++u) s0[u] = 0.0, s1[u] = 0.0;
    // two segments (the two-stage split copies, ts_stage0): the product formed where the entry is
    // added.  Measured at 400^3 (levels 5-6, the longest groups) 8-10 % faster than the form below,
    // which holds every gather in flight at once (86 VGPRs against 64: 5 waves per SIMD)
    for (int k = k0 + lane; k < k1 && S == 2; k += 64 * U) {
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
            if (k + 64 * t >= k1) break;
            const double p = a[t] * fetch((int)(q[t] >> kMergeShift));
            const unsigned key = q[t] & ((1u << kMergeShift) - 1);
#pragma unroll
            for (int u = 0; u < G; ++u) {
                s0[u] += key == (unsigned)u ? p : 0.0;
                s1[u] += key == (unsigned)(8 + u) ? p : 0.0;
            }
        }
    }
    for (int k = k0 + lane; k < k1 && S == 1; k += 64 * U) {
        unsigned q[U];
        double a[U], xv[U];
        // keys and values loaded unconditionally (clamped into the group), every x gather issued
        // before any product is formed: with the multiply under each gather's condition the
        // compiler waited for each gather in turn.  An entry past the group adds +0.0 to row 0's
        // accumulator -- an exact identity, as the +0.0s every entry adds to the other rows'
        // accumulators (no accumulator is ever -0.0)
#pragma unroll
        for (int t = 0; t < U; ++t) {
            const int kk = k + 64 * t, kc = kk < k1 ? kk : k1 - 1;
            q[t] = mk[kc];
            a[t] = mv[kc];
        }
#pragma unroll
        for (int t = 0; t < U; ++t) xv[t] = k + 64 * t < k1 ? fetch((int)(q[t] >> kMergeShift)) : 0.0;
#pragma unroll
        for (int t = 0; t < U; ++t) {
            const bool live = k + 64 * t < k1;
            const double p = live ? a[t] * xv[t] : 0.0;
            const unsigned key = live ? q[t] & ((1u << kMergeShift) - 1) : 0u;
#pragma unroll
            for (int u = 0; u < G; ++u) {
                s0[u] += key == (unsigned)u ? p : 0.0;
                if (S == 2) s1[u] += key == (unsigned)(8 + u) ? p : 0.0;
            }
        }
    }
#pragma unroll
    for (int u = 0; u < G; ++u)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            s0[u] += __shfl_xor(s0[u], off, 64);
            if (S == 2) s1[u] += __shfl_xor(s1[u], off, 64);
        }
}

// Merged groups per 256-thread workgroup: W waves per group (W = 1, 2 or 4, DevCSR::mg_W), so
// 4 / W groups per workgroup; the waves of a group take consecutive 1/W shares of its entries
// (merged_sums each), then thread t < (4/W) G reports (group t / G, row t % G): the W partials
// added in wave order (fixed: deterministic).  Returns false for threads without a row.
// red: 8G doubles of LDS.  Must be reached by every thread of the block.
template <int G, int S, class Fetch>
__device__ __forceinline__ bool merged_block(const int *__restrict__ gp, int ng, int W, const unsigned *__restrict__ mk,
                                             const double *__restrict__ mv, Fetch fetch, double *red, int &g_out,
                                             int &u_out, double &t0, double &t1)
{
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, gpb = 4 / W;
    const int g = xcd_bid() * gpb + w / W, part = w % W;
    double s0[G], s1[G];
    if (g < ng) {
        const int k0 = gp[g], k1 = gp[g + 1], len = k1 - k0, per = (len + W - 1) / W;
        merged_sums<G, S>(k0 + min(len, part * per), k0 + min(len, (part + 1) * per), mk, mv, fetch, s0, s1);
    } else {
#pragma unroll
        for (int u = 0; u < G; ++u) s0[u] = 0.0, s1[u] = 0.0;
    }
    if (lane == 0)
#pragma unroll
        for (int u = 0; u < G; ++u) {
            red[(w * 2) * G + u] = s0[u];
            if (S == 2) red[(w * 2 + 1) * G + u] = s1[u];
        }
    __syncthreads();
    const int t = threadIdx.x;
    if (t >= gpb * G) return false;
    const int gi = t / G, u = t % G, gg = xcd_bid() * gpb + gi;
    if (gg >= ng) return false;
    double a0 = red[((gi * W) * 2) * G + u], a1 = S == 2 ? red[((gi * W) * 2 + 1) * G + u] : 0.0;
    for (int v = 1; v < W; ++v) {
        a0 += red[((gi * W + v) * 2) * G + u];
        if (S == 2) a1 += red[((gi * W + v) * 2 + 1) * G + u];
    }
    g_out = gg, u_out = u, t0 = a0, t1 = a1;
    return true;
}

}  // namespace sss
