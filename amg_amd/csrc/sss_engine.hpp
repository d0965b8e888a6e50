// sss_engine.hpp — internal declarations of the gfx950 engine (not part of any public ABI).
//
// Layout in HBM (DESIGN.md §Data layout): every level keeps the reference's CSR arrays
// (int32 row_ptr / col_idx, fp64 val) for A, P and R, plus b, x, wp (fp64, length n_l) and
// the C/F marker.  Index arrays are int32 exactly as in SSS_main.h:95-105; all arithmetic is
// fp64 without contraction (-ffp-contract=off) so the parity kernels reproduce the host
// reference bit for bit.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <string>
#include <functional>
#include <memory>
#include <cstdio>
#include <thread>
#include <vector>

#include "../../include/sss_hip.h"

// roctx ranges (amg_amd/host/sss_util.c; rocprofv3 --marker-trace)
extern "C" void sss_trace_push(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
extern "C" void sss_trace_pop(void);
namespace sss {
struct TraceRange {
    template <class... Args>
    explicit TraceRange(const char *fmt, Args... a) { sss_trace_push(fmt, a...); }
    ~TraceRange() { sss_trace_pop(); }
    TraceRange(const TraceRange &) = delete;
    TraceRange &operator=(const TraceRange &) = delete;
};
}  // namespace sss

extern "C" void sss_huge_hint(void *p, size_t bytes);   // amg_amd/host/sss_util.c

namespace sss {

constexpr int kBlock = 256;        // threads per workgroup for streaming kernels (4 waves)
constexpr int kTileEntries = 2048; // CSR entries staged in LDS per SpMV row block (24 KiB)
constexpr int kMaxLevels = max_AMG_LVL;

int hip_fail(hipError_t e, const char *what, const char *file, int line);
#define SSS_HIP(call)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (call);                                                          \
        if (e_ != hipSuccess) return ::sss::hip_fail(e_, #call, __FILE__, __LINE__);    \
    } while (0)

template <class T>
inline T *dev_alloc(size_t count)
{
    void *p = nullptr;
    if (count == 0) count = 1;
    if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) return nullptr;
    return static_cast<T *>(p);
}
inline void dev_free(void *p)
{
    if (p) (void)hipFree(p);
}

// Host array without value-initialisation (the upload builders overwrite every element, and
// zero-filling gigabyte arrays on one thread was a visible share of the upload time).
template <class T>
struct HostBuf {
    std::unique_ptr<T[]> p;
    size_t n = 0;
    void resize(size_t m)
    {
        p.reset(m ? new T[m] : nullptr);
        sss_huge_hint(p.get(), m * sizeof(T));   // large, untouched: transparent huge pages
        n = m;
    }
    T *data() { return p.get(); }
    const T *data() const { return p.get(); }
    size_t size() const { return n; }
    T &operator[](size_t i) { return p[i]; }
    const T &operator[](size_t i) const { return p[i]; }
};

// Persistent host worker pool for the upload-time data preparation (sss_spmv.hip): the workers
// are started once and reused, so a parallel loop costs a wake-up instead of thread creation
// (h2d alone issued one loop per 32 MiB chunk).  Up to 8 callers' loops at once, idle workers
// joining any of them; a loop issued from a worker runs inline on it.
int host_pool_threads();
void host_thread_background();   // lower the calling thread's CPU priority (SSS_HOST_NICE)
bool host_pool_run(const std::function<void()> &work);   // false: caller runs inline

// Host-side data preparation at upload: fn(lo, hi) over [0, n) in chunks of `grain` items taken
// from a shared counter by the pool's threads and the caller (the .hip units are compiled
// without OpenMP).
template <class Fn>
void parallel_chunks(int n, int grain, Fn fn)
{
    if (n <= 0) return;
    if (n <= grain || host_pool_threads() <= 1) {
        fn(0, n);
        return;
    }
    std::atomic<int> next{0};
    std::function<void()> work = [&]() {
        for (;;) {
            const int lo = next.fetch_add(grain);
            if (lo >= n) return;
            fn(lo, std::min(n, lo + grain));
        }
    };
    if (!host_pool_run(work)) work();
}

// Upload phase timer: SSS_HIP_TIMING=2 prints each mark's elapsed time on stderr.
struct PhaseTimer {
    const char *what;
    bool on;
    double t;
    std::vector<std::pair<const char *, double>> marks;
    static double now()
    {
        return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    explicit PhaseTimer(const char *w) : what(w)
    {
        const char *e = getenv("SSS_HIP_TIMING");
        on = e && atoi(e) >= 2;
        t = now();
    }
    void mark(const char *name)
    {
        if (!on) return;
        const double t1 = now();
        marks.emplace_back(name, t1 - t);
        t = t1;
    }
    ~PhaseTimer()
    {
        if (!on || marks.empty()) return;
        std::string s;
        char buf[96];
        for (auto &m : marks) {
            snprintf(buf, sizeof(buf), " %s %.3f", m.first, m.second);
            s += buf;
        }
        fprintf(stderr, "[sss_hip]     %s:%s\n", what, s.c_str());
    }
};

// In-place prefix sum of a[1..n] (a[0] given): a[i + 1] += a[i] over chunks on the pool.
inline void parallel_prefix(int *a, int n)
{
    constexpr int kC = 1 << 16;
    const int nc = (n + kC - 1) / kC;
    if (nc <= 1) {
        for (int i = 0; i < n; ++i) a[i + 1] += a[i];
        return;
    }
    std::vector<long long> tot((size_t)nc + 1, 0);
    parallel_chunks(nc, 1, [&](int c0, int c1) {
        for (int c = c0; c < c1; ++c) {
            long long t = 0;
            for (int i = c * kC; i < std::min(n, (c + 1) * kC); ++i) t += a[i + 1];
            tot[(size_t)c + 1] = t;
        }
    });
    tot[0] = a[0];
    for (int c = 0; c < nc; ++c) tot[(size_t)c + 1] += tot[c];
    parallel_chunks(nc, 1, [&](int c0, int c1) {
        for (int c = c0; c < c1; ++c) {
            long long run = tot[c];
            for (int i = c * kC; i < std::min(n, (c + 1) * kC); ++i) run += a[i + 1], a[i + 1] = (int)run;
        }
    });
}

// Host -> device copy through pinned staging buffers (sss_spmv.hip); returns 0 or an error code.
int h2d(void *dst, const void *src, size_t bytes);

// CSR matrix resident in HBM, plus its CSR-adaptive row blocking for SpMV.
struct DevCSR {
    int n = 0, ncols = 0, nnz = 0;
    int *rp = nullptr, *ci = nullptr;
    double *v = nullptr;
    int nblk = 0;          // SpMV row blocks
    int *blk = nullptr;    // block -> first row (nblk + 1 entries)
    int2 *bk = nullptr;    // block -> {first row, first entry} (nblk + 1): one load, no rp[blk[.]] chain
    const int2 *h_bk = nullptr;   // host copy of bk (the byte ledger's block -> rows / entries)
    int split_row = -1;    // class split row the blocks were cut at (-1: none)
    int split_blk = 0;     // index of the block starting at split_row
    bool wave_rows = false;  // long rows: wave-per-row kernels (avg nnz/row >= kWaveRowMin)
    int ngrid = 0;           // workgroups of one SpMV launch (size of a per-block partial array)
    // Column-sorted tile staging (kEncSortedTiles; bitwise-neutral): each staging segment of the
    // blocking -- a block's entries, or a kTileEntries chunk of a longer row -- stored sorted by
    // column as pk = cluster << 31 | (col - base[cluster]) << kTileShift | (stored-order position
    // in the segment), pv = values; pb[block] = {base0, base1}.  A block's columns form at most two
    // clusters (cut at their widest gap: the F and C halves of a relabeled level, own rows and
    // ghosts), each spanning < 2^kTileColBits columns, or the matrix keeps stored order (pk null).
    // Products land in LDS at their stored position, so every row chain keeps the reference's
    // order; neighbouring rows' gathers of the same x lines coalesce (measured 1.4-1.7x on the
    // coarse levels of 7-pt 400^3, tools/lab_rows.hip).
    unsigned *pk = nullptr;
    double *pv = nullptr;
    int2 *pb = nullptr;
    // kEncFreeOrder on a long-row matrix (>= free_row_min() entries per row on average): rows summed
    // in a fixed tree order, deterministic but NOT the reference order.  ci/v then hold each row
    // (or each of its two segments [rp, seg) / [seg, rp+1)) column-sorted for the wave-per-row
    // kernels (64 lane-strided sums, xor-shuffle reduction) ...
    bool vec_rows = false;
    bool rows_sorted = false;  // vec_rows: ci/v hold each row (segment) column-sorted (else stored order)
    // ... and on a short-row matrix of a free-order level, the rows longer than one tile (a hub
    // row of an irregular operator) are tree-summed chunk by chunk by the whole workgroup instead
    // of chained by one thread (block_tree_sum; the short rows keep the stored order)
    bool tree_long = false;
    // ... and, for matrices with enough rows to fill the chip in groups (merge_group_size), a
    // merged copy: G consecutive rows' entries merged into one column-sorted list, packed
    // col << 4 | segment << 3 | row-in-group (segment: 0, or 1 for [seg, rp+1) of two-segment rows).  One wave sums a group lane-strided with one accumulator per
    // row; neighbouring rows share most columns, so a wave's 64 gathers touch ~G x fewer x lines
    // (the long-row levels are bound by the L2->CU line rate of those gathers, not by HBM).
    // Dictionary tiles (kEncDict; bitwise-neutral): every staging segment column-sorted (as the
    // sorted tiles), each entry a 32-bit code  value index << 19 | offset index << 11 | position
    // in the segment  into its block's dictionaries of distinct column offsets col - row (<= 256)
    // and distinct value bit patterns (<= 256): 4 B per entry instead of 12, gathers still in
    // column order.  dv_pd[block] = {offset base, offset count, value base, value count}.  Built
    // only when every block qualifies (7-pt Poisson level 0: 7 offsets and 2 values per block).
    // Value-dictionary sorted tiles (kEncDict, when the offsets do not fit a dictionary but every
    // block has <= 256 distinct values -- a relabeled Galerkin level): the sorted tiles' pk/pb with
    // a 1-byte value index dv_vi per slot into the block's value dictionary instead of pv: 5 B per
    // entry.  dv_code stays null, dv_pd[block].y = 0, pv is not uploaded.
    // Dictionary ELL (kEncDict, tried first; stencil levels: every row <= 32 entries, every block
    // <= 31 column offsets and <= 8 values -- 7-pt level 0): row r's entries in stored order as
    // ell_w one-byte codes  value index << 5 | offset index  at dv_ell[r * ell_w] (0xFF pads), into
    // the block dictionaries dv_pd/dv_dd/dv_vd.  One thread per row, no LDS staging, no row_ptr:
    // ell_w bytes per row (8 for 7-pt) instead of 12 per entry.  pk and dv_code stay null.
    unsigned char *dv_ell = nullptr;
    int ell_w = 0;
    // A rectangular operator's dictionary ELL may store its offsets against a per-row base column
    // (the row's first column) instead of the row index: dv_ell_base[r] (null: the row index).  A
    // restriction's rows follow the next level's F-first relabeling, so col - row drifts across a
    // block while col - (first col) repeats the stencil.
    int *dv_ell_base = nullptr;
    // Column ELL (kEncDict, when the offsets do not fit a 1-byte dictionary but every row has at
    // most 32 entries, every 256-row block few enough distinct values and the columns fit the code -- the Galerkin
    // level of a stencil, 7-pt level 1: 19 entries per row): row r's entries in stored order as
    // xell_w 32-bit codes  value index << xell_shift | column  at dv_xell[r * xell_w] (0xFFFFFFFF pads) into
    // the block value dictionaries dv_pd[block].z/.w -> dv_vd.  One thread per row, no LDS staging:
    // 4 B per entry (as the value-dictionary tiles' 5) without the tile's staging barrier and its
    // 2048-entry blocks (~108 rows of a 19-entry level): blocks are 256 rows.
    unsigned *dv_xell = nullptr;
    int xell_w = 0;
    int xell_shift = 0;   // column bits S of a code (value index << S | column); >= 23
    long long stream_bytes = 0;   // bytes of the stored format one tile-path SpMV streams (no vectors)
    unsigned *dv_code = nullptr;
    unsigned char *dv_vi = nullptr;
    int4 *dv_pd = nullptr;
    int *dv_dd = nullptr;
    double *dv_vd = nullptr;
    int mg_G = 0;              // 0: no merged copy
    int mg_ng = 0;             // groups
    int mg_W = 4;              // waves per group (1, 2 or 4): 4 / mg_W groups per workgroup
    int *mg_gp = nullptr;      // per group: first entry (mg_ng + 1)
    bool mg_two = false;       // two-segment rows
    unsigned *mg_k = nullptr;
    double *mg_v = nullptr;
};
constexpr int kMergeShift = 4;           // segment + row-in-group bits of a merged entry (G <= 8)
constexpr int kTileShift = 11;           // log2(kTileEntries)
constexpr int kTileColBits = 20;         // column offset bits of a packed sorted-tile entry
// Offsets >= kTileDiagMark mark a diagonal entry: offset - kTileDiagMark = its row in the block (so
// its column is the block's first row + that), and the staging also keeps its raw value in LDS.
constexpr unsigned kTileDiagMark = (1u << kTileColBits) - 256;
static_assert((1 << kTileShift) == kTileEntries, "tile packing");
static_assert(1 + kTileColBits + kTileShift == 32, "tile packing");
// kEncMergedOnly: the matrix is only ever read through its merged copy when it gets one (the
// two-stage split copies, launch_ts_*), so its CSR arrays need not be column-sorted
// kEncXell: the column ELL may replace the tile storage (its own 256-row blocking)
enum { kEncSortedTiles = 1, kEncFreeOrder = 2, kEncDict = 4, kEncMergedOnly = 8, kEncXell = 16,
       kEncEll = 32,      // kEncEll: the one-byte dictionary ELL only (also rectangular; no dictionary tiles)
       kEncEllBase = 64 };   // kEncEllBase: a rectangular matrix's dictionary ELL with per-row bases (dv_ell_base)
// split >= 0 forces a row-block boundary at that row (the F|C class boundary of a relabeled level);
// enc: kEnc* flags; seg (kEncFreeOrder only, optional): per row, the absolute CSR position that
// splits the row into two independently summed segments (two-stage [N_i | L_i] rows).
int devcsr_upload(DevCSR &d, const SSS_MAT &h, int split = -1, int enc = 0, const int *seg = nullptr);
// encoding flags a hierarchy level uses for its matrices under the options o, and for its
// transfer operators P_l, R_l
int level_encoding(const sss_hip_opts &o);
int transfer_encoding(const sss_hip_opts &o);
int restriction_encoding(const sss_hip_opts &o);
void devcsr_free(DevCSR &d);
int build_row_blocks(const int *h_rp, int n, std::vector<int> &blk, int split = -1);
// *host (optional): a new[]-allocated host copy (DevCSR::h_bk, released by devcsr_free)
int upload_block_bounds(int2 **dst, const std::vector<int> &blk, const int *h_rp, const int2 **host = nullptr);
int wave_row_min();
int free_row_min();
// Re-upload a free-order matrix's CSR rows column-sorted (one uploaded kEncMergedOnly whose
// merged copy turned out not to be its only reader).
int devcsr_sort_rows(DevCSR &d, const SSS_MAT &h, const int *seg = nullptr);
// Device-side builders of the free-order formats (sss_build.hip; SSS_HIP_GPU_BUILD=0 keeps the
// host builders): merged row groups from the resident stored-order CSR, and the in-place column
// sort of each row (segment).  Results are the host builders' bit for bit.
bool device_builders_on();
int merged_build_device(DevCSR &d, const int *h_seg);
int sort_rows_device(DevCSR &d, const int *h_seg);
struct DevDict;
DevDict devdict(const DevCSR &A, int blo);   // the matrix's dictionary tiles, block numbers from blo
// the tile kernels stage from a dictionary (either kind): instantiate them with DICT = true
inline bool has_dict(const DevCSR &A)
{
    return A.dv_code != nullptr || A.dv_vi != nullptr || A.dv_ell != nullptr || A.dv_xell != nullptr;
}
// Storage argument K of the tile kernels: 0 plain or sorted tiles, 1 dictionary tiles (either kind),
// 8 / 16 / 32 dictionary ELL of that row width, kXell + W column ELL of row width W (8/16/20/24/32/40).
constexpr int kXell = 256;
// row blocks per workgroup of a launch over storage K (dictionary ELL: 2, measured against 1 and 4)
constexpr int rows_per_wg(int K) { return K >= kXell ? 1 : K >= 8 ? 2 : 1; }
// f(std::integral_constant<int, K>) with the storage argument K of A
template <class F>
inline void with_tile_kind(const DevCSR &A, F f)
{
    if (A.dv_xell) {
        if (A.xell_w == 8) f(std::integral_constant<int, kXell + 8>{});
        else if (A.xell_w == 16) f(std::integral_constant<int, kXell + 16>{});
        else if (A.xell_w == 20) f(std::integral_constant<int, kXell + 20>{});
        else if (A.xell_w == 24) f(std::integral_constant<int, kXell + 24>{});
        else if (A.xell_w == 32) f(std::integral_constant<int, kXell + 32>{});
        else f(std::integral_constant<int, kXell + 40>{});
    } else if (A.dv_ell) {
        if (A.ell_w == 8) f(std::integral_constant<int, 8>{});
        else if (A.ell_w == 16) f(std::integral_constant<int, 16>{});
        else f(std::integral_constant<int, 32>{});
    } else if (has_dict(A)) {
        f(std::integral_constant<int, 1>{});
    } else {
        f(std::integral_constant<int, 0>{});
    }
}

// ---- stored-format byte ledger (bench.py `vcycle_stored`, tools/level_breakdown.py) -------------
// While a ledger is installed on the calling thread (sss_hip_cycle_bytes: one eager walk of the
// cycle with launches enqueued as usual), every launch helper adds the bytes its kernel reads and
// writes: the stored format of the rows it covers (codes, dictionaries, values, row bounds --
// DevCSR::stream_bytes pro rata: by rows for the ELL formats, by entries otherwise), 8 B per covered
// row for every row vector it streams (b, y read and/or written, divisors, P), and the x it gathers
// counted once per covered row (8 B x covered rows x ncols / n).  Slot kMaxLevels is the outer
// residual + norm, kMaxLevels + 1 the coarsest solve.
struct ByteLedger {
    double bytes[kMaxLevels + 2] = {};
    int slot = 0;
};
extern thread_local ByteLedger *g_ledger;
inline void ledger_add(double b)
{
    if (g_ledger) g_ledger->bytes[g_ledger->slot] += b;
}
inline bool ledger_on() { return g_ledger != nullptr; }
double matrix_bytes(const DevCSR &A, int blo, int bhi);   // stored bytes of row blocks [blo, bhi)
double matrix_bytes_rows(const DevCSR &A, int lo, int hi);   // ... of rows [lo, hi) (block granularity)
inline double xgather_bytes(const DevCSR &A, double rows) { return A.n ? 8.0 * rows * A.ncols / A.n : 0.0; }

// ---- hierarchy internals shared with the distributed engine (sss_hier.hip) ------------------
// A hierarchy over mg->cg[0 .. num_levels); its L[0] is global level `level_base` (smoother
// kinds follow the global level); `stream` = nullptr creates a private stream.
sss_hip_hier *hier_create_impl(const SSS_AMG *mg, const sss_hip_opts *o, int level_base, hipStream_t stream);
double *hier_vec(sss_hip_hier *h, int level, int which);
const std::vector<int> &hier_perm(sss_hip_hier *h, int level);   // new -> old (empty: identity)
int level_kind_of(const sss_hip_opts &o, int global_level);
// The stall word of the hierarchy's one-launch GS passes: read (and cleared) with a sync -- 0 or
// ERROR_MISC with an "### ERROR" line on stderr; re-pointed to an owner's word (distributed tail).
int hier_stall_check(sss_hip_hier *h);
unsigned *hier_err_word(sss_hip_hier *h);
bool hier_coarse_on_device(sss_hip_hier *h);   // the coarsest solve is device-only (explicit inverse)
void hier_set_err_word(sss_hip_hier *h, unsigned *err);
// two-stage inner steps of a global level of `rows` rows and `nnz` entries (the whole level's, on
// every rank of a partitioned one)
int level_inner_of(const sss_hip_opts &o, int global_level, long long rows, long long nnz);

// y <- op(A x) on `stream` (see SSS_HIP_SPMV_*).  `partial` (optional, RESID only): one
// sum-of-squares of the written y per row block, for a deterministic fused norm.
int launch_spmv(const DevCSR &A, int op, double alpha, const double *x, const double *b, double *y,
                int cap, double *partial, hipStream_t stream);
// x[lo + q] += e[col[q]] for q < m, with the AMXPY epilogue's arithmetic of a row holding one 1.0.
int launch_prolong_inject(int m, int lo, const int *col, const double *e, double *x, hipStream_t stream);
// As launch_spmv, tile path only, over the row blocks [blo, bhi) of A (partial indexed by block).
int launch_spmv_range(const DevCSR &A, int blo, int bhi, int op, double alpha, const double *x, const double *b,
                      double *y, double *partial, hipStream_t stream);
inline int launch_spmv_blocks(const DevCSR &A, int nblk, int op, double alpha, const double *x, const double *b,
                              double *y, double *partial, hipStream_t stream)
{
    return launch_spmv_range(A, 0, nblk, op, alpha, x, b, y, partial, stream);
}

// ---- smoother schedules -------------------------------------------------------------------
// One-launch exact GS-CF pass (sss_gs_persist.hip): engine 0 = one launch per DAG depth,
// 1 = chip-wide dataflow ("flow"), 2 = single-CU ("cu").
struct GsPersist {
    int engine = 0;
    int lo = 0, hi = 0;                 // the pass's contiguous rows
    int G = 64;                         // flow: lanes per row (64 / G rows of one depth per ticket)
    bool overlap = false;               // flow: the chain runs while pending granules are polled (long rows)
    bool natural = false, desc = false; // natural-order GS (x = t * d), descending row order
    int nchunks = 0, grid = 0;
    int *ck = nullptr;                  // flow, short rows: chunk -> first position (nchunks + 1)
    int *h_off = nullptr;               // cu: depth offsets (depth + 1)
    unsigned *ctl = nullptr;            // epoch, ticket, exit count, error
    unsigned *err = nullptr;            // where a stall is reported: ctl's error word, or the
                                        // hierarchy's (smoother_set_err)
    int spin = 0;                       // polls before a waiting wave gives up (< 0: test hook)
    unsigned long long *gran = nullptr; // flow: two {epoch, half of x_i} granules per row
};
// Every sweep's F and C passes of one exact GS-CF smoother call as ONE dataflow launch
// (sss_gs_persist.hip, "fused" engine): nodes (row, sweep) in fused-DAG depth order.
struct GsFused {
    int engine = 0;                     // 1: built
    int sweeps = 0;                     // the call's sweeps this plan is for
    int n = 0, split = 0;               // rows; F rows [0, split), C rows [split, n)
    int G = 64;                         // lanes per row
    bool overlap = false;               // the chain runs while pending granules are polled
    int shards = 8;                     // ticket counters (SSS_HIP_FUSED_SHARDS; 1 = one device-wide)
    int depth = 0, nchunks = 0, grid = 0;
    int *ck = nullptr;                  // chunk -> first position in nodes (nchunks + 1)
    int *nodes = nullptr;               // sweep * n + row, by fused depth
    // Sweep 0 of a call on a zero iterate (the pre-smoother of a level the descent just cleared):
    // each row's entries whose version-0 value it would read are exactly zero, so with finite
    // values (and b_i != -0.0) their products can be dropped from the stored-order chain without
    // changing a bit -- rows of only the entries read at a later version, in stored order.
    int *rp0 = nullptr, *ci0 = nullptr;
    double *v0 = nullptr;
    unsigned *ctl = nullptr;            // epoch, ticket, exit count, error
    unsigned *err = nullptr;
    int spin = 0;
    unsigned long long *gran = nullptr; // two {epoch << 4 | version, half of x_i} granules per row
};
struct PassSchedule {          // rows of one class (F or C), grouped by DAG depth
    int depth = 0;
    std::vector<int> h_off;    // depth + 1 offsets into rows
    int *rows = nullptr;       // device
    int nrows = 0;
    int max_width = 0;
    // Row-compacted CSR of this class (rows ascending) with CSR-adaptive blocking: used when
    // the pass has no intra-class couplings (depth 1) or for C/F-Jacobi.
    bool compact = false;
    // Contiguous class (relabeled level, F rows first): the pass is rows [lo, hi) = blocks [blo, bhi)
    // of the level matrix itself; no copy.
    bool range = false;
    int lo = 0, hi = 0, blo = 0, bhi = 0;
    double *y2 = nullptr;      // second inner-iterate buffer (two-stage)
    // Two-stage GS-CF (sss_smooth.hip): the pass's rows with their off-diagonal entries reordered
    // to [N_i | L_i] (L_i: same class, j < i; both in stored order), the split positions, the
    // L-only rows, and P_i = b_i - sum_{N_i} a_ij x_j of the current pass.
    DevCSR ts_nl, ts_lo;
    int *ts_split = nullptr;
    double *ts_P = nullptr;
    DevCSR sub;
    int *map = nullptr;        // local row -> global row
    double *y = nullptr;       // Jacobi: new values of this class, scattered after the pass
    GsPersist gp;              // exact GS with depth > 1: one launch per pass when set up
};
// natural: x_i = t * d (unguarded, d = 1 / a_ii); desc: rows taken in descending order (the
// rows a row waits for are the same-pass rows above it)
int gs_persist_build(PassSchedule &ps, const SSS_MAT &A, int lo, int hi, bool long_rows, bool natural = false,
                     bool desc = false);
void gs_persist_free(PassSchedule &ps);
int gs_persist_run(const PassSchedule &ps, const DevCSR &A, const double *b, double *x, const double *deff,
                   hipStream_t s);
int gs_persist_error(const PassSchedule &ps, unsigned *out);
// cls: per row 1 = C
int gs_fused_build(GsFused &f, const SSS_MAT &A, const DevCSR *dA, const PassSchedule *pass, const int *cls,
                   int sweeps);
int gs_fused_run(const GsFused &f, const DevCSR &A, const double *b, double *x, const double *d_first,
                 const double *d_later, bool x_zero, hipStream_t s);
void gs_fused_free(GsFused &f);
// *out = the fused engine's stall word (0 when the plan has no fused engine); cleared if set and clear
int gs_fused_error(const GsFused &f, unsigned *out, bool clear);
struct SmootherPlan;
// Report the one-launch passes' stalls into *err (a word of the owning hierarchy).
void smoother_set_err(SmootherPlan &sp, unsigned *err);
// *out = 1.0 if *err is set else 0.0, and *err cleared (one thread on stream s).
int launch_err_flag(unsigned *err, double *out, hipStream_t s);
struct SmootherPlan {
    int kind = SSS_HIP_SMOOTH_EXACT;
    // Natural-order GS (SSS_amg_smoother_gs, Solve/SSS_smooth.c:90-137: cf_order = 0 or no C/F
    // marker): pass[0] = the rows ascending (pre-smoother), pass[1] = descending (post), each one
    // class; x_i = t * d with d = 1 / a_ii carried across rows (d_first/d_later per direction:
    // d_first, d_later for pass[0]; nd_first, nd_later for pass[1]).
    bool natural = false;
    double *nd_first = nullptr, *nd_later = nullptr;
    PassSchedule pass[2];      // [0] = F pass (mark != 1), [1] = C pass (mark == 1)
    GsFused fz;                // exact GS-CF: all passes of a call in one launch (when built)
    double *d_first = nullptr; // effective divisor for the first sweep of a call
    double *d_later = nullptr; // ... for later sweeps (aliases d_first when all rows have a diagonal)
    int *cls = nullptr;        // per row: 1 if mark == 1 else 0
    bool long_rows = false;    // wave-per-row kernels
    int *diag_pos = nullptr;   // range passes: CSR position of each row's diagonal (-1: none)
    int inner = 0;             // two-stage GS-CF inner steps (kind == JACOBI, range passes only)
    // No-copy C/F-Jacobi (kind == JACOBI, both passes range, class split at csplit): a pass writes
    // its class's new values into the other of {x, x2} and later passes read each class from where
    // its current values are; an even number of writes per class (the default 2 sweeps) leaves
    // everything back in x.
    double *x2 = nullptr;
    int csplit = 0;
    // The last class pass of a call (C, rows [split_row, n)) can also write the residual
    // r = b - A x of its rows (ResidFuse): exact GS with depth-1 range passes (a red-black level),
    // every row with exactly one diagonal, no long-row block among the C blocks.
    bool fuse_resid = false;
    // The F pass has depth 1 (no F-F coupling) and divides every F row by |d| > 1e-20 in every
    // sweep: it overwrites x_F from C values only, so whatever x_F held before is dead (the
    // prolongation into F rows before a post-smoother can be skipped).
    bool f_overwritten = false;
    // Every row has exactly one diagonal entry, so every sweep's divisor is the row's own diagonal:
    // tile passes over a sorted-tile matrix read it from the staged tile instead of d_first/d_later.
    bool own_diag = false;
    // The outer residual's F half may also compute the next call's first F pass (relax_range<3>):
    // fuse_resid and f_overwritten hold and no F block is a long row.  smoother_run's pre_f then
    // skips that pass and lets the first C pass read the F values from pre_f.
    bool pend_ok = false;
    // Every value of A is finite: a pass over a zero iterate reduces to t = b (zero_first_pass).
    bool finite = false;
};
// Residual fused into the smoother's last pass: r[i] = b[i] - sum_k a_ik x_k (stored order from
// 0.0, x after the pass) for the C rows, and their per-block sums of squares into partial[block]
// when partial is given; the caller then forms the F rows' residual (blocks [0, split_blk)).
struct ResidFuse {
    double *r = nullptr;
    double *partial = nullptr;
    bool done = false;         // set by smoother_run when it fused
};
// contiguous: mark is relabeled so class F occupies rows [0, nF) and class C rows [nF, n), and A was
// uploaded with a block split at nF (its DevCSR is passed to allow range passes).
// gcls (distributed levels, A has ghost columns >= num_rows): per ghost, its class if it is owned by
// a lower rank (a "lower" column for the two-stage form), else -1.
// Distributed levels: called before every class pass with x (exchange its ghosts), and after each
// two-stage stage with the stage's full-length work vector; w0/w1 are full-length (own + ghost) work
// vectors the two-stage form then writes its iterates into.
// split (optional): refresh vec's ghosts while launching the row blocks [blo, bhi) of the level
// matrix -- launch(b0, b1) for the blocks that read no ghost while the halo is in flight, then for
// the others (or everything after a plain exchange).  Each row is computed exactly as in one launch.
struct PassHooks {
    void *ctx = nullptr;
    int (*exchange)(void *ctx, double *vec) = nullptr;
    double *w0 = nullptr, *w1 = nullptr;
    std::function<int(double *vec, int blo, int bhi, const std::function<void(int, int)> &launch)> split;
};
int smoother_build(SmootherPlan &sp, const SSS_MAT &A, const int *mark, int kind, const DevCSR *dA = nullptr,
                   int inner = 0, const int *gcls = nullptr, int enc = 0);
// Natural-order GS over the rows [lo, hi) (both directions; see SmootherPlan::natural).
int smoother_build_natural(SmootherPlan &sp, const SSS_MAT &A, int lo, int hi);
// Where a pass reads its x values from: columns < split from f, the others from c.  The no-copy
// C/F-Jacobi form keeps each class's current values in x or in the plan's second vector x2.
struct XSrc {
    const double *f, *c;
    int split;
    __device__ __forceinline__ double operator()(int j) const { return j < split ? f[j] : c[j]; }
};
inline XSrc xsrc_of(const double *x) { return XSrc{x, x, 0x7fffffff}; }
void launch_ts_stage0(const DevCSR &M, int lo, const int *split, const double *b, XSrc x, const double *deff,
                      double *P, double *y, hipStream_t s);
void launch_ts_inner(const DevCSR &M, int lo, const double *deff, const double *P, const double *ycols, int col_off,
                     const double *ykeep, double *y, hipStream_t s);
void smoother_free(SmootherPlan &sp);
int smoother_run(const SmootherPlan &sp, const DevCSR &A, const double *b, double *x, int sweeps,
                 hipStream_t stream, const PassHooks *hooks = nullptr, ResidFuse *rf = nullptr,
                 const double *pre_f = nullptr, bool x_zero = false, bool post = false);
// r = b - A x over the F rows (+ per-block partials) and pend = the F pass's GS values from this x
// (SmootherPlan::pend_ok).
int launch_f_residual_pending(const SmootherPlan &sp, const DevCSR &A, const double *b, const double *x, double *r,
                              double *partial, double *pend, hipStream_t s);

// ---- reductions ----------------------------------------------------------------------------
// Deterministic sum of `n` partials -> *out (device); optionally sqrt.  `partials` must hold
// n + kFinalScratch doubles: the tail is scratch for the first of two reduction stages.
constexpr int kFinalScratch = 256;
int launch_final_sum(double *partials, int n, double *out, bool take_sqrt, hipStream_t s);

// ---- BLAS-1 for the preconditioned CG (sss_blas.hip) ---------------------------------------
// dot: partial must hold 1024 + kFinalScratch doubles; *out on the device.
int launch_dot(int n, const double *a, const double *b, double *partial, double *out, hipStream_t s);
// y += sign * (*num / *den) * x
int launch_axpy_ratio(int n, const double *num, const double *den, double sign, const double *x, double *y,
                      hipStream_t s);
// p = z + ((*num - *numold) / *den) * p   (numold null: *num / *den)
int launch_xpby_ratio(int n, const double *num, const double *numold, const double *den, const double *z, double *p,
                      hipStream_t s);

// ---- coarse solvers ------------------------------------------------------------------------
struct CoarseDirect {
    int n = 0;
    double *inv = nullptr;     // row-major explicit inverse
};
int coarse_direct_build(CoarseDirect &cd, const SSS_MAT &A, hipStream_t stream);
void coarse_direct_free(CoarseDirect &cd);
int coarse_direct_apply(const CoarseDirect &cd, const double *b, double *x, hipStream_t stream);

struct CoarseKrylov;           // reference CG(beta==1)+GMRES(30) on device
CoarseKrylov *coarse_krylov_create(const DevCSR &A, int row_cap, hipStream_t stream);
void coarse_krylov_destroy(CoarseKrylov *k);
int coarse_krylov_solve(CoarseKrylov *k, const DevCSR &A, const double *b, double *x, double ctol,
                        hipStream_t stream);

}  // namespace sss
