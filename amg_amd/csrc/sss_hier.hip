// sss_hier.hip — HBM mirror of an SSS_AMG hierarchy and the device V-cycle.
//
// The V/W-cycle control flow of SSS_amg_cycle (Solve/SSS_cycle.cu:848-967) is static given
// cycle_type, so the host walks it and enqueues kernels on one stream without synchronising:
//   descent  : smoother_pre(l); wp_l = b_l - A_l x_l (one fused kernel, SSS_cycle.cu:916-917);
//              b_{l+1} = R_l wp_l (:921); x_{l+1} = 0 (:929)
//   coarsest : SSS_amg_coarest_solve (:933) -> Krylov (parity) or explicit inverse (direct)
//   ascent   : x_l += P_l x_{l+1} (:942); smoother_post(l) (:958)
// The outer residual r = b - A0 x and ||r|| (Solve/SSS_SOLVE.c:59-64) are one fused kernel
// writing per-block sums of squares plus a one-block deterministic reduction; the 8-byte
// norm is the only per-iteration device->host transfer.
#include "sss_engine.hpp"
#include "sss_tail.hpp"

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>

#include <chrono>

#include <cmath>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

using namespace sss;

struct sss_hip_hier {
    int nl = 0;
    SSS_AMG_PARS pars{};
    sss_hip_opts opts{};
    hipStream_t stream = nullptr;
    struct Level {
        DevCSR A, P, R;
        double *b = nullptr, *x = nullptr, *wp = nullptr;
        // the C rows of P as injections (each one stored 1.0): their coarse columns, for the
        // prolongation into the C rows only (hb_level_pr); null = the tile path
        int *pinj = nullptr;
        SmootherPlan sm;
        // Relabeling (new -> old) of this level's unknowns: F points first, then C points, each in
        // ascending original order; empty = identity (coarsest level, or relabeling off).
        std::vector<int> perm;
    } L[kMaxLevels];
    std::vector<double> stage;   // host staging for permuted vector transfers
    int level_base = 0;          // global level index of L[0] (a tail of a distributed hierarchy)
    // hybrid smoother on a level 0 whose classes are not independent sets: two-stage GS-CF there
    bool hybrid0_two_stage = false;
    bool own_stream = true;
    int coarse_mode = SSS_HIP_COARSE_DIRECT;
    CoarseDirect direct;
    CoarseKrylov *krylov = nullptr;
    double *partial = nullptr;   // per-row-block partial sums for the level-0 norm
    double *d_norm = nullptr;    // [0] ||r||, [1] 1.0 if a one-launch GS pass stalled since the last read
    double *h_norm = nullptr;    // pinned mirror of d_norm
    unsigned *d_err = nullptr;   // stall word of every one-launch GS pass of the hierarchy
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // hipGraph replay of the cycle: segments between host-steered coarse solves (a null exec
    // marks "run the Krylov coarse solve here"); the residual-norm tail has its own graph.
    std::vector<hipGraphExec_t> cycle_steps;
    bool cycle_graph_ready = false;
    hipGraphExec_t resid_exec = nullptr;
    // ResidFuse on level 0 (SmootherPlan::fuse_resid): the cycle's last C pass leaves the C rows of
    // r = b - A0 x in wp and their block partials in `partial`; the residual norm then only forms
    // the F rows.  Valid from the end of a cycle until level-0 x or b is touched by anything else.
    bool resid_c_ready = false;
    hipGraphExec_t resid_f_exec = nullptr;
    // SmootherPlan::pend_ok on level 0: the residual norm's F half also produced the next cycle's
    // first F pass (pend_f, F rows); valid while level-0 x and b are untouched.
    bool pending_f = false;
    double *pend_f = nullptr;
    std::vector<hipGraphExec_t> cycle_steps_p;   // cycle graph variant that consumes pend_f
    bool cycle_graph_ready_p = false;
    int cycle_kernels = 0, cycle_kernels_p = 0;   // kernel launches per cycle in the captured graphs
    // AMG-preconditioned CG (sss_hip_pcg): level-0 work vectors, dot partials, device scalars
    double *pcg_v = nullptr;     // 7 vectors of n0: b, x, r, z, p, q, r_old
    double *pcg_part = nullptr;
    double *pcg_s = nullptr;     // device scalars
    double *pcg_h = nullptr;     // pinned host mirror
    TailPlan tail;               // the small coarse levels as one single-workgroup launch (sss_tail.hip)
    // per-level timing of an eager cycle (sss_hip_time_levels): an event after each step of the
    // walk, tagged with the level the step belonged to
    std::vector<hipEvent_t> lev_ev;
    std::vector<int> lev_tag;
    int lev_n = 0;
};

static int env_int(const char *name, int dflt)
{
    const char *s = getenv(name);
    return (s && *s) ? atoi(s) : dflt;
}

extern "C" void sss_hip_opts_default(sss_hip_opts *o)
{
    std::memset(o, 0, sizeof(*o));
    o->device = env_int("SSS_HIP_DEVICE", -1);
    o->smoother = SSS_HIP_SMOOTH_EXACT;
    o->coarse = SSS_HIP_COARSE_KRYLOV;
    o->row_cap = env_int("SSS_HIP_ROWCAP", 0);
    o->use_graph = env_int("SSS_HIP_GRAPH", 1);
    o->verbose = env_int("SSS_HIP_VERBOSE", 0);
    o->relabel = env_int("SSS_HIP_RELABEL", 1);
    o->inner = env_int("SSS_HIP_INNER", 1);
    o->inner_from = env_int("SSS_HIP_INNER_FROM", 2);
    o->inner_long = env_int("SSS_HIP_INNER_LONG", 1);
    o->sorted_tiles = env_int("SSS_HIP_SORTED_TILES", 1);
    o->sum_order = env_int("SSS_HIP_SUM_ORDER", 0);
    o->formats = -1;
    if (const char *f = getenv("SSS_HIP_FORMATS")) {
        const std::string v(f);
        if (v == "full") o->formats = 0;
        else if (v == "lean") o->formats = 1;
    }
    if (const char *s = getenv("SSS_HIP_SMOOTHER")) {
        std::string v(s);
        if (v == "hybrid") o->smoother = SSS_HIP_SMOOTH_HYBRID;
        else if (v == "jacobi") o->smoother = SSS_HIP_SMOOTH_JACOBI;
    }
    if (const char *s = getenv("SSS_HIP_COARSE")) {
        std::string v(s);
        if (v == "direct") o->coarse = SSS_HIP_COARSE_DIRECT;
    }
}

extern "C" int sss_hip_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int sss_hip_mem_info(size_t *free_bytes, size_t *total_bytes)
{
    size_t f = 0, t = 0;
    SSS_HIP(hipMemGetInfo(&f, &t));
    *free_bytes = f;
    *total_bytes = t;
    return 0;
}

static int level_smoother_kind(const sss_hip_opts &o, int l)
{
    if (o.smoother == SSS_HIP_SMOOTH_JACOBI) return SSS_HIP_SMOOTH_JACOBI;
    if (o.smoother == SSS_HIP_SMOOTH_HYBRID && l > 0) return SSS_HIP_SMOOTH_JACOBI;
    return SSS_HIP_SMOOTH_EXACT;
}

// two-stage inner steps of level l (0 = plain C/F-Jacobi there, or not a C/F-Jacobi level)
// rows / nnz: the whole (global) level's, so every rank of a partitioned level decides alike
static int level_inner(const sss_hip_opts &o, int l, long long rows, long long nnz)
{
    if (level_smoother_kind(o, l) != SSS_HIP_SMOOTH_JACOBI || l < o.inner_from || o.inner <= 0) return 0;
    const bool long_rows = rows > 0 && nnz >= (long long)SSS_HIP_LONG_ROW_MIN * rows;
    return o.inner + (long_rows ? std::max(0, o.inner_long) : 0);
}
int sss::level_kind_of(const sss_hip_opts &o, int l) { return level_smoother_kind(o, l); }
int sss::level_encoding(const sss_hip_opts &o)
{
    // plain CSR tiles only: asked for, or (auto) the exact smoother -- its cycle waits on the GS-CF
    // chains (7-pt 400^3: ~1.2 s per cycle), and the formats' host builders were ~40 % of its mirror
    if (o.formats == 1 || (o.formats < 0 && o.smoother == SSS_HIP_SMOOTH_EXACT))
        return o.sum_order == 1 ? kEncFreeOrder : 0;
    // dictionary tiles (kEncDict) are offered for the level matrices A_l; uploads of P, R and the
    // two-stage split copies mask them out (their column offsets are not row-relative)
    const char *dz = getenv("SSS_HIP_DICT");
    const int dict = (dz && *dz == '0') ? 0 : kEncDict;
    return (o.sorted_tiles ? kEncSortedTiles : 0) | (o.sum_order == 1 ? kEncFreeOrder : 0) | dict | (dict ? kEncXell : 0);
}
int sss::level_inner_of(const sss_hip_opts &o, int l, long long rows, long long nnz)
{
    return level_inner(o, l, rows, nnz);
}
// P_l and R_l: the level matrices' encodings without the dictionary tiles (measured at 7-pt 400^3:
// 22.15 -> 22.25 ms per V-cycle with them, level-0 prolongation 255 -> 325 us -- P's F rows have
// 1-8 irregular columns, so the per-tile dictionaries rarely shrink a row and the extra
// indirection costs more than the 3 bytes saved per entry); the column ELL is offered to them.
int sss::transfer_encoding(const sss_hip_opts &o) { return level_encoding(o) & ~kEncDict; }
// R_l: as transfer_encoding, plus the one-byte dictionary ELL with per-row base columns (a
// restriction's rows follow the next level's F-first order, so offsets col - row drift across a
// block while col - first col repeats; tools/fmt_probe.py reports the formats each operator got).
int sss::restriction_encoding(const sss_hip_opts &o)
{
    const char *bz = getenv("SSS_HIP_ELL_BASE");   // 0: no per-row-based dictionary ELL for R
    int enc = transfer_encoding(o);
    if ((level_encoding(o) & kEncDict) && !(bz && *bz == '0')) enc |= kEncEllBase;
    return enc;
}

// Are the C and the F points of A each an independent set (no off-diagonal coupling inside a
// class)?  Then exact GS-CF has no chains: each class pass is one C/F-Jacobi pass (7-pt level 0).
static bool classes_independent(const SSS_MAT &A, const int *mark)
{
    std::atomic<int> ok{1};
    parallel_chunks(A.num_rows, 1 << 14, [&](int lo, int hi) {
        for (int i = lo; i < hi && ok; ++i) {
            const bool ci = mark[i] == 1;
            for (int k = A.row_ptr[i]; k < A.row_ptr[i + 1]; ++k) {
                const int j = A.col_idx[k];
                if (j != i && (mark[j] == 1) == ci) {
                    ok = 0;
                    return;
                }
            }
        }
    });
    return ok != 0;
}

// per-level smoother of this hierarchy (level_smoother_kind/level_inner with the hybrid level-0
// rule applied)
static int hier_kind(const sss_hip_hier *h, int gl)
{
    if (gl == 0 && h->hybrid0_two_stage) return SSS_HIP_SMOOTH_JACOBI;
    return level_smoother_kind(h->opts, gl);
}
static int hier_inner(const sss_hip_hier *h, int gl, const SSS_MAT &A)
{
    if (gl == 0 && h->hybrid0_two_stage) return std::max(1, h->opts.inner);
    return level_inner(h->opts, gl, A.num_rows, A.num_nnzs);
}

// Natural-order GS (SSS_amg_smoother_pre/post with cf_order = 0, Solve/SSS_smooth.c:171-176,
// 256-260) on the levels the reference would smooth by GS
static bool natural_level(const sss_hip_hier *h, int gl)
{
    return h->pars.cf_order == 0 && h->pars.smoother == SSS_SM_GS && hier_kind(h, gl) == SSS_HIP_SMOOTH_EXACT;
}

static void hier_release(sss_hip_hier *h)
{
    if (!h) return;
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (int l = 0; l < h->nl; ++l) {
        auto &L = h->L[l];
        devcsr_free(L.A);
        devcsr_free(L.P);
        devcsr_free(L.R);
        dev_free(L.pinj);
        L.pinj = nullptr;
        dev_free(L.b);
        dev_free(L.x);
        dev_free(L.wp);
        smoother_free(L.sm);
    }
    for (auto g : h->cycle_steps)
        if (g) (void)hipGraphExecDestroy(g);
    if (h->resid_exec) (void)hipGraphExecDestroy(h->resid_exec);
    if (h->resid_f_exec) (void)hipGraphExecDestroy(h->resid_f_exec);
    for (hipGraphExec_t g : h->cycle_steps_p)
        if (g) (void)hipGraphExecDestroy(g);
    tail_free(h->tail);
    dev_free(h->pend_f);
    dev_free(h->pcg_v);
    dev_free(h->pcg_part);
    dev_free(h->pcg_s);
    if (h->pcg_h) (void)hipHostFree(h->pcg_h);
    coarse_direct_free(h->direct);
    coarse_krylov_destroy(h->krylov);
    dev_free(h->partial);
    dev_free(h->d_norm);
    dev_free(h->d_err);
    if (h->h_norm) (void)hipHostFree(h->h_norm);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->stream && h->own_stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

// ---- class-contiguous relabeling ------------------------------------------------------------
// Each level's unknowns are renumbered F-first (mark != 1), C-second, keeping the original order
// inside each class.  Every kernel computes a row from the same entries in the same CSR order, GS
// sweeps visit each class in the same relative order, and the coarsest level (Krylov dot products)
// keeps its labels, so the iterates are bitwise those of the unrelabeled hierarchy.  What changes
// is the memory layout: every smoother pass is a contiguous row range of the level matrix, the
// x values it gathers (the other class) are contiguous too, and it writes a dense half of x.
struct RelabeledCSR {   // owns the arrays an SSS_MAT view points into
    HostBuf<int> rp;
    HostBuf<int> ci;
    HostBuf<double> v;
    SSS_MAT view(int nrows, int ncols)
    {
        SSS_MAT m;
        m.num_rows = nrows;
        m.num_cols = ncols;
        m.num_nnzs = (int)ci.size();
        m.row_ptr = rp.data();
        m.col_idx = ci.data();
        m.val = v.data();
        return m;
    }
};

// B = A with rows taken in order rperm (new -> old; empty = identity) and columns renamed by
// cinv (old -> new; empty = identity); entry order inside a row is unchanged.
static void relabel_csr(const SSS_MAT &A, const std::vector<int> &rperm, const std::vector<int> &cinv, RelabeledCSR &B)
{
    const int n = A.num_rows;
    B.rp.resize((size_t)n + 1);
    B.rp[0] = 0;
    parallel_chunks(n, 1 << 16, [&](int lo, int hi) {
        for (int i = lo; i < hi; ++i) {
            const int o = rperm.empty() ? i : rperm[i];
            B.rp[(size_t)i + 1] = A.row_ptr[o + 1] - A.row_ptr[o];
        }
    });
    parallel_prefix(B.rp.data(), n);
    B.ci.resize((size_t)B.rp[n]);
    B.v.resize((size_t)B.rp[n]);
    parallel_chunks(n, 1 << 15, [&](int lo, int hi) {
        for (int i = lo; i < hi; ++i) {
            const int o = rperm.empty() ? i : rperm[i];
            int q = B.rp[i];
            for (int k = A.row_ptr[o]; k < A.row_ptr[o + 1]; ++k, ++q) {
                B.ci[q] = cinv.empty() ? A.col_idx[k] : cinv[A.col_idx[k]];
                B.v[q] = A.val[k];
            }
        }
    });
}

// ---- construction ---------------------------------------------------------------------------
// The mirror is built level by level: begin (stream, events), then per level the relabeling, A_l
// with its smoother plan, and P_l / R_l (which need the next level's relabeling), then finish
// (coarse solver, graph decision).  hier_create_impl runs a set-up hierarchy's level steps side by
// side on a few host threads; sss_hip_setup_create runs them on a worker thread while SSS_amg_setup
// is still coarsening the later levels (a level is handed over once the setup has moved past it).
struct HierBuild {
    sss_hip_hier *h = nullptr;
    const SSS_AMG *mg = nullptr;
    std::vector<std::vector<int>> inv = std::vector<std::vector<int>>(kMaxLevels);
    std::vector<int> nF = std::vector<int>(kMaxLevels, -1);
    std::atomic<const char *> err{nullptr};
    bool timing = getenv("SSS_HIP_TIMING") != nullptr;   // per-level upload phases on stderr
};

static bool hb_fail(HierBuild &b, const char *what)
{
    if (!b.err) b.err = what;
    return false;
}

static bool hb_begin(HierBuild &b, const SSS_AMG *mg, const sss_hip_opts *o, int level_base, hipStream_t stream)
{
    if (sss_hip_device_count() <= 0) {
        fprintf(stderr, "### ERROR: no HIP device available for the AMG solve phase\n");
        return false;
    }
    auto *h = b.h = new sss_hip_hier();
    b.mg = mg;
    h->nl = 0;
    h->pars = mg->pars;
    if (o) h->opts = *o;
    else sss_hip_opts_default(&h->opts);
    if (h->opts.device >= 0 && hipSetDevice(h->opts.device) != hipSuccess) return hb_fail(b, "device");
    h->level_base = level_base;
    if (stream) {
        h->stream = stream;
        h->own_stream = false;
    } else if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        return hb_fail(b, "stream");
    }
    if (hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess) return hb_fail(b, "events");
    return true;
}

// F|C relabeling of a level that is not the coarsest (the coarsest keeps the identity)
static void hb_perm(HierBuild &b, int l)
{
    sss_hip_hier *h = b.h;
    const SSS_AMG *mg = b.mg;
    // hybrid: exact GS-CF on level 0 only where it is chain-free (its cost is then that of
    // C/F-Jacobi); a level 0 with same-class couplings (27-pt, irregular operators) would run the
    // level-scheduled chains every sweep -- there the two-stage form takes its place
    if (l == 0 && h->opts.smoother == SSS_HIP_SMOOTH_HYBRID && h->level_base == 0 && mg->cg[0].cfmark.d &&
        mg->cg[0].cfmark.n >= mg->cg[0].A.num_rows && mg->pars.cf_order != 0)
        h->hybrid0_two_stage = !classes_independent(mg->cg[0].A, mg->cg[0].cfmark.d);
    const SSS_AMG_COMP &C = mg->cg[l];
    const int n = C.A.num_rows;
    if (!C.cfmark.d || C.cfmark.n < n) return;
    // two-stage levels need contiguous classes; otherwise follow opts.relabel
    const int gl = h->level_base + l;
    const bool two_stage = hier_inner(h, gl, C.A) > 0;
    if (natural_level(h, gl)) return;   // the natural order is the stored row order
    if (!two_stage && !(h->opts.relabel == 1 || (h->opts.relabel == 2 && gl > 0))) return;
    auto &perm = h->L[l].perm;
    perm.reserve(n);
    for (int i = 0; i < n; ++i)
        if (C.cfmark.d[i] != 1) perm.push_back(i);
    b.nF[l] = (int)perm.size();
    for (int i = 0; i < n; ++i)
        if (C.cfmark.d[i] == 1) perm.push_back(i);
    b.inv[l].resize(n);
    auto &iv = b.inv[l];
    parallel_chunks(n, 1 << 16, [&](int lo, int hi) {
        for (int i = lo; i < hi; ++i) iv[perm[i]] = i;
    });
}

// A_l (+ its smoother plan unless coarsest) and the level vectors
static bool hb_level_a(HierBuild &b, int l, bool coarsest)
{
    TraceRange tr("mirror level %d: A + smoother plan", l);
    sss_hip_hier *h = b.h;
    const SSS_AMG_COMP &C = b.mg->cg[l];
    auto &L = h->L[l];
    const int n = C.A.num_rows;
    const bool rl = !L.perm.empty();
    const double t_a = PhaseTimer::now();
    double t_rel = t_a, t_up = t_a, t_sm = t_a;
    // the coarsest operator only feeds the coarse solver: stored order there.  On a two-stage level
    // the relaxation reads the split copies, and the level matrix's own free-order products go
    // through its merged copy (residual) or are order-free (zero-first pass): no sorted rows needed
    int enc = !coarsest ? level_encoding(h->opts) : (level_encoding(h->opts) & kEncSortedTiles);
    if (!coarsest && hier_kind(h, h->level_base + l) == SSS_HIP_SMOOTH_JACOBI && hier_inner(h, h->level_base + l, C.A) > 0)
        enc |= kEncMergedOnly;
    if (rl) {
        RelabeledCSR B;
        relabel_csr(C.A, L.perm, b.inv[l], B);
        SSS_MAT Av = B.view(n, C.A.num_cols);
        t_rel = PhaseTimer::now();
        if (devcsr_upload(L.A, Av, b.nF[l], enc)) return hb_fail(b, "upload A");
        t_up = PhaseTimer::now();
        HostBuf<int> mark;
        mark.resize((size_t)n);
        parallel_chunks(n, 1 << 16, [&](int lo, int hi) {
            for (int i = lo; i < hi; ++i) mark[i] = C.cfmark.d[L.perm[i]];
        });
        if (smoother_build(L.sm, Av, mark.data(), hier_kind(h, h->level_base + l), &L.A,
                           hier_inner(h, h->level_base + l, C.A), nullptr, enc))
            return hb_fail(b, "smoother plan");
        if (L.sm.inner == 0 && devcsr_sort_rows(L.A, Av)) return hb_fail(b, "upload A");   // plain passes read A's rows
        t_sm = PhaseTimer::now();
    } else {
        if (devcsr_upload(L.A, C.A, -1, enc)) return hb_fail(b, "upload A");
        if (!coarsest && natural_level(h, h->level_base + l)) {
            if (smoother_build_natural(L.sm, C.A, 0, n)) return hb_fail(b, "smoother plan");
        } else if (!coarsest && smoother_build(L.sm, C.A, C.cfmark.d, hier_kind(h, h->level_base + l), nullptr, 0,
                                               nullptr, enc)) {
            return hb_fail(b, "smoother plan");
        }
        if (devcsr_sort_rows(L.A, C.A)) return hb_fail(b, "upload A");   // (no two-stage plan here)
        t_rel = t_up = t_a;
        t_sm = PhaseTimer::now();
    }
    if (b.timing)
        fprintf(stderr, "[sss_hip] upload level %d: relabel %.2f s, A %.2f s, smoother plan %.2f s\n", l,
                rl ? t_rel - t_a : 0.0, rl ? t_up - t_rel : t_sm - t_a, rl ? t_sm - t_up : 0.0);
    L.b = dev_alloc<double>((size_t)n);
    L.x = dev_alloc<double>((size_t)n);
    L.wp = dev_alloc<double>((size_t)n);
    if (!L.b || !L.x || !L.wp) return hb_fail(b, "vectors");
    if (hipMemset(L.b, 0, sizeof(double) * n) != hipSuccess || hipMemset(L.x, 0, sizeof(double) * n) != hipSuccess ||
        hipMemset(L.wp, 0, sizeof(double) * n) != hipSuccess)
        return hb_fail(b, "memset");
    return true;
}

// P_l and R_l: rows / columns follow the relabelings of levels l and l + 1 (hb_perm of l + 1 has
// run, or l + 1 is the coarsest)
static bool hb_level_pr(HierBuild &b, int l)
{
    TraceRange tr("mirror level %d: P, R", l);
    sss_hip_hier *h = b.h;
    const SSS_AMG_COMP &C = b.mg->cg[l];
    auto &L = h->L[l];
    const bool rl = !L.perm.empty();
    const auto &pc = h->L[l + 1].perm;
    // a prolongation applied to the C rows only (SmootherPlan::f_overwritten: one stored entry each)
    // keeps the tiles -- the column ELL would read a padded row of codes per entry (7-pt level 0,
    // 258 -> 289 us per V-cycle)
    const int tenc = transfer_encoding(h->opts);
    const int penc = L.sm.f_overwritten ? (tenc & ~kEncXell) : tenc;
    const double t0 = PhaseTimer::now();
    if (rl || !pc.empty()) {
        PhaseTimer pt("P/R");
        RelabeledCSR P, R;
        relabel_csr(C.P, L.perm, b.inv[l + 1], P);
        pt.mark("relabel P");
        relabel_csr(C.R, pc, b.inv[l], R);
        pt.mark("relabel R");
        // P's rows follow the level's F|C relabeling: blocks split there too, so a
        // prolongation can be limited to the C rows (SmootherPlan::f_overwritten)
        const SSS_MAT Pv = P.view(C.P.num_rows, C.P.num_cols);
        if (devcsr_upload(L.P, Pv, rl ? b.nF[l] : -1, penc) ||
            devcsr_upload(L.R, R.view(C.R.num_rows, C.R.num_cols), -1, restriction_encoding(h->opts)))
            return hb_fail(b, "upload P/R");
        // the prolongation into the C rows only (f_overwritten): when every C row of P is one stored
        // 1.0, its columns alone (SSS_HIP_INJECT=0: the tile path)
        const char *iz = getenv("SSS_HIP_INJECT");
        if (rl && L.sm.f_overwritten && b.nF[l] > 0 && !(iz && *iz == '0')) {
            const int n = Pv.num_rows, lo = b.nF[l];
            std::vector<int> col((size_t)(n - lo));
            std::atomic<bool> ok{true};
            parallel_chunks(n - lo, 1 << 16, [&](int a, int e) {
                for (int q = a; q < e && ok; ++q) {
                    const int k = Pv.row_ptr[lo + q];
                    if (Pv.row_ptr[lo + q + 1] != k + 1 || Pv.val[k] != 1.0) ok = false;
                    else col[q] = Pv.col_idx[k];
                }
            });
            if (ok) {
                L.pinj = dev_alloc<int>(col.size());
                if (!L.pinj || h2d(L.pinj, col.data(), sizeof(int) * col.size())) return hb_fail(b, "upload P injection");
            }
        }
    } else if (devcsr_upload(L.P, C.P, -1, penc) || devcsr_upload(L.R, C.R, -1, restriction_encoding(h->opts))) {
        return hb_fail(b, "upload P/R");
    }
    if (b.timing) fprintf(stderr, "[sss_hip] upload level %d: P/R %.2f s\n", l, PhaseTimer::now() - t0);
    return true;
}

// The V-cycle's tail (sss_tail.hip): the coarsest levels whose passes are all tiny, run as one
// single-workgroup launch.  A level qualifies when it is smoothed by the no-copy two-stage
// C/F-Jacobi form on the tile paths (rows of at most one tile, so every row sum is a stored-order
// chain) and is small (<= 4,096 rows and <= SSS_HIP_TAIL_NNZ nonzeros in A, default 16,384); the coarsest level needs the explicit
// inverse and <= 256 rows.  The tail is the longest such run above the coarsest level (level 0
// never: its residual and smoothers have their own fused forms).  SSS_HIP_TAIL=0: no tail.
static int max_row(const SSS_MAT &M)
{
    int mx = 0;
    for (int i = 0; i < M.num_rows; ++i) mx = std::max(mx, M.row_ptr[i + 1] - M.row_ptr[i]);
    return mx;
}
static int tail_build(sss_hip_hier *h, const SSS_AMG *mg)
{
    h->tail = TailPlan();
    const char *tz = getenv("SSS_HIP_TAIL");
    const int nl = h->nl;
    if ((tz && *tz == '0') || nl < 3 || h->level_base != 0 || h->coarse_mode != SSS_HIP_COARSE_DIRECT ||
        h->direct.n > 256 || (h->pars.cycle_type > 1))
        return 0;
    const char *tn = getenv("SSS_HIP_TAIL_NNZ");
    const int tail_nnz = (tn && *tn) ? atoi(tn) : 16384;
    auto ok = [&](int l) {
        const auto &L = h->L[l];
        const SmootherPlan &sp = L.sm;
        if (sp.kind != SSS_HIP_SMOOTH_JACOBI || sp.inner < 1 || !sp.x2 || sp.natural) return false;
        // one workgroup streams ~8K entries per microsecond: past ~16K nonzeros a pass is slower
        // in it than as its own launch across the chip (the stand-in's level 7, 169K nonzeros,
        // took 4.5 ms in the tail against 0.18 ms per V-cycle as launches)
        if (L.A.n > 4096 || L.A.nnz > tail_nnz) return false;
        if (L.A.wave_rows || L.A.vec_rows || L.P.wave_rows || L.P.vec_rows || L.R.wave_rows || L.R.vec_rows) return false;
        for (const auto &ps : sp.pass)
            if (ps.nrows > 0 && (!ps.range || ps.ts_nl.vec_rows || ps.ts_nl.wave_rows || ps.ts_lo.vec_rows || ps.ts_lo.wave_rows))
                return false;
        const SSS_AMG_COMP &C = mg->cg[l];
        return max_row(C.A) <= kTileEntries && max_row(C.P) <= kTileEntries && max_row(C.R) <= kTileEntries;
    };
    int from = nl - 1;
    while (from - 1 >= 1 && ok(from - 1)) --from;
    if (from >= nl - 1) return 0;
    std::vector<TailLevel> lv;
    for (int l = from; l + 1 < nl; ++l) {
        const auto &L = h->L[l];
        const SmootherPlan &sp = L.sm;
        TailLevel t;
        t.n = L.A.n;
        t.nc = h->L[l + 1].A.n;
        t.b = L.b, t.x = L.x, t.x2 = sp.x2, t.wp = L.wp;
        t.deff = sp.d_first;
        t.csplit = sp.csplit, t.inner = sp.inner, t.pre = h->pars.pre_iter, t.post = h->pars.post_iter;
        t.finite = sp.finite ? 1 : 0;
        for (int c = 0; c < 2; ++c) {
            const PassSchedule &ps = sp.pass[c];
            TailPass &tp = t.pass[c];
            tp.lo = ps.nrows > 0 ? ps.lo : 0;
            tp.hi = ps.nrows > 0 ? ps.hi : 0;
            tp.nrp = ps.ts_nl.rp, tp.nci = ps.ts_nl.ci, tp.nv = ps.ts_nl.v, tp.split = ps.ts_split;
            tp.lrp = ps.ts_lo.rp, tp.lci = ps.ts_lo.ci, tp.lv = ps.ts_lo.v, tp.P = ps.ts_P;
        }
        // ledger: per sweep each class pass streams its [N | L] rows and `inner` times its L rows
        // (+ 40 B of vectors per row each), then the residual, R and P
        const int sweeps = h->pars.pre_iter + h->pars.post_iter;
        for (int c = 0; c < 2; ++c)
            if (sp.pass[c].nrows > 0)
                h->tail.ledger_bytes += sweeps * ((double)sp.pass[c].ts_nl.stream_bytes + 40.0 * sp.pass[c].nrows +
                                                  sp.inner * ((double)sp.pass[c].ts_lo.stream_bytes + 40.0 * sp.pass[c].nrows));
        h->tail.ledger_bytes += (double)L.A.stream_bytes + (double)L.R.stream_bytes + (double)L.P.stream_bytes +
                                32.0 * L.A.n + 16.0 * t.nc;
        t.arp = L.A.rp, t.aci = L.A.ci, t.av = L.A.v;
        t.rrp = L.R.rp, t.rci = L.R.ci, t.rv = L.R.v;
        t.prp = L.P.rp, t.pci = L.P.ci, t.pv = L.P.v;
        lv.push_back(t);
    }
    const auto &Cl = h->L[nl - 1];
    h->tail.ledger_bytes += 8.0 * h->direct.n * (double)h->direct.n + 16.0 * h->direct.n;
    h->tail.inv = h->direct.inv;
    h->tail.nc = h->direct.n;
    h->tail.cb = Cl.b;
    h->tail.cx = Cl.x;
    if (int rc = tail_upload(h->tail, lv)) return rc;
    h->tail.from = from;
    return 0;
}

static sss_hip_hier *hb_finish(HierBuild &b)
{
    sss_hip_hier *h = b.h;
    const SSS_AMG *mg = b.mg;
    auto fail = [&](const char *what) {
        fprintf(stderr, "### ERROR: sss_hip_hier_create: %s\n", what);
        hier_release(h);
        b.h = nullptr;
        return (sss_hip_hier *)nullptr;
    };
    if (b.err) return fail(b.err);
    h->partial = dev_alloc<double>((size_t)h->L[0].A.ngrid + kFinalScratch);
    if (h->nl > 1 && h->L[0].sm.pend_ok) {
        h->pend_f = dev_alloc<double>((size_t)std::max(h->L[0].sm.pass[0].hi, 1));
        if (!h->pend_f) return fail("pending F pass buffer");
    }
    h->d_norm = dev_alloc<double>(2);
    h->d_err = dev_alloc<unsigned>(1);
    if (!h->partial || !h->d_norm || !h->d_err || hipHostMalloc((void **)&h->h_norm, 2 * sizeof(double)) != hipSuccess)
        return fail("norm buffers");
    if (hipMemset(h->d_err, 0, sizeof(unsigned)) != hipSuccess || hipMemset(h->d_norm, 0, 2 * sizeof(double)) != hipSuccess)
        return fail("norm buffers");
    for (int l = 0; l + 1 < h->nl; ++l) smoother_set_err(h->L[l].sm, h->d_err);

    const SSS_MAT &Ac = mg->cg[h->nl - 1].A;
    h->coarse_mode = h->opts.coarse;
    if (h->coarse_mode == SSS_HIP_COARSE_DIRECT && Ac.num_rows > 20000) h->coarse_mode = SSS_HIP_COARSE_KRYLOV;
    if (h->coarse_mode == SSS_HIP_COARSE_DIRECT) {
        if (coarse_direct_build(h->direct, Ac, h->stream)) return fail("coarse inverse");
    } else {
        h->krylov = coarse_krylov_create(h->L[h->nl - 1].A, h->opts.row_cap, h->stream);
        if (!h->krylov) return fail("coarse Krylov workspace");
    }
    if (tail_build(h, mg)) return fail("tail levels");
    if (hipStreamSynchronize(h->stream) != hipSuccess) return fail("sync");
    // Graph replay only pays for, and is only robust with, a modest node count: the exact
    // smoother on deep coarse levels issues one launch per DAG depth (~10^5 per cycle).
    long long launches = 0;
    for (int l = 0; l + 1 < h->nl; ++l) {
        const auto &sm = h->L[l].sm;
        long long per_sweep = 0;
        for (const auto &ps : sm.pass)
            per_sweep += ps.nrows == 0 ? 0
                         : ps.compact ? (sm.kind == SSS_HIP_SMOOTH_JACOBI ? 2 + sm.inner : 1)
                         : ps.gp.engine ? 1 : ps.depth;
        launches += per_sweep * (h->pars.pre_iter + h->pars.post_iter) + 4;
    }
    if (launches > 4096) h->opts.use_graph = 0;
    if (h->opts.verbose) {
        for (int l = 0; l < h->nl; ++l)
            fprintf(stderr, "[sss_hip] level %d: n=%d nnz=%d blocks=%d dagF=%d dagC=%d kind=%d gs engine F/C=%d/%d\n", l,
                    h->L[l].A.n, h->L[l].A.nnz, h->L[l].A.nblk, h->L[l].sm.pass[0].depth, h->L[l].sm.pass[1].depth,
                    h->L[l].sm.kind, h->L[l].sm.pass[0].gp.engine, h->L[l].sm.pass[1].gp.engine);
    }
    b.h = nullptr;
    return h;
}


// Setup and mirror construction overlapped: SSS_amg_setup (host, reference semantics) runs on the
// calling thread; each time it completes a level, a worker thread relabels and uploads the levels
// whose neighbourhood is final -- A_l and its smoother plan once level l is known not to be the
// coarsest, P_l / R_l once level l + 1's relabeling is known.  The worker's host loops share the
// CPUs with the setup's OpenMP regions, and its uploads run while the setup's serial RS passes
// (Setup/SSS_coarsen.c:294-498) keep one core busy.  Results are those of SSS_amg_setup followed by
// sss_hip_hier_create.
namespace {
// The mirror's level tasks: A(l) = relabel + A_l + smoother plan (once the setup has moved past level
// l), PR(l) = P_l / R_l (once A(l) has finished and level l + 1's relabeling is known).  While the
// setup runs, one background worker takes them in order; once it has returned, the calling thread
// and two more threads take whatever is runnable, so the levels the
// setup produced last -- each an independent plan build -- are uploaded side by side.
struct Pipeline {
    HierBuild b;
    std::mutex mu;
    std::condition_variable cv;
    int done = 0;         // levels the setup has moved past (final, not the coarsest)
    bool finished = false;
    int device = 0;
    double t_setup_end = 0, t_worker_end = 0;
    int a_next = 0, pr_next = 0, busy = 0;
    std::vector<char> a_fin = std::vector<char>(kMaxLevels, 0), perm_fin = std::vector<char>(kMaxLevels, 0);
    // under mu: the next runnable task (+l: A(l - 1), -l: PR(l - 1)), 0 = none now
    int claim()
    {
        if (b.err) return 0;
        // PR(l): A(l) done, and level l + 1's relabeling known (or l + 1 the coarsest, which keeps
        // the identity; the calling thread uploads that last PR after the setup)
        if (pr_next + 1 < done && a_fin[pr_next] && perm_fin[pr_next + 1]) return -(++pr_next);
        if (a_next < done) return ++a_next;
        return 0;
    }
    void run(int task)
    {
        if (task > 0) {
            const int l = task - 1;
            hb_perm(b, l);
            {
                std::lock_guard<std::mutex> lk(mu);
                perm_fin[l] = 1;
            }
            cv.notify_all();
            hb_level_a(b, l, false);
            std::lock_guard<std::mutex> lk(mu);
            a_fin[l] = 1;
        } else {
            hb_level_pr(b, -task - 1);
        }
    }
    // take tasks until none is left; the background worker also waits for the setup's progress
    void loop(bool background)
    {
        for (;;) {
            int t;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] {
                    if (b.err) return true;
                    if (claim_peek()) return true;
                    return !background ? busy == 0 : finished && busy == 0;
                });
                t = claim();
                if (!t) {
                    if (b.err || busy == 0) break;
                    continue;
                }
                ++busy;
            }
            run(t);
            {
                std::lock_guard<std::mutex> lk(mu);
                --busy;
            }
            cv.notify_all();
        }
        cv.notify_all();
    }
    bool claim_peek() const
    {
        return !b.err && ((pr_next + 1 < done && a_fin[pr_next] && perm_fin[pr_next + 1]) || a_next < done);
    }
    void worker()
    {
        (void)hipSetDevice(device);
        host_thread_background();
        loop(true);
        t_worker_end = PhaseTimer::now();
    }
};
}   // namespace

// The levels the task runner did not take -- the last non-coarsest level's P/R (its next level, the
// coarsest, keeps the identity) and the coarsest operator -- then the hierarchy's final assembly.
static sss_hip_hier *pipeline_finish(Pipeline &P, const SSS_AMG *mg)
{
    HierBuild &b = P.b;
    const int nl = mg->num_levels;
    if (!b.err) {
        int a_done = 0, pr_done = 0;
        for (int l = 0; l < nl; ++l)
            if (b.h->L[l].A.rp) a_done = l + 1;
        for (int l = 0; l + 1 < nl; ++l)
            if (b.h->L[l].P.rp) pr_done = l + 1;
        for (int l = a_done; l + 1 < nl && !b.err; ++l) hb_perm(b, l), hb_level_a(b, l, false);
        for (int l = pr_done; l + 1 < nl && !b.err; ++l) hb_level_pr(b, l);
        if (!b.err && !b.h->L[nl - 1].A.rp) hb_level_a(b, nl - 1, true);
    }
    return hb_finish(b);
}

static void pipeline_hook(void *ctx, const SSS_AMG *mg, int done, int final)
{
    (void)mg;
    auto *P = static_cast<Pipeline *>(ctx);
    {
        std::lock_guard<std::mutex> lk(P->mu);
        P->done = done;
        if (final) P->finished = true;
    }
    P->cv.notify_all();
}

extern "C" sss_hip_hier *sss_hip_setup_create(SSS_AMG *mg, SSS_MAT *A, SSS_AMG_PARS *pars, const sss_hip_opts *o,
                                              double *times)
{
    if (!mg || !A || !pars) return nullptr;
    const double t0 = PhaseTimer::now();
    Pipeline P;
    // the mirror's begin needs mg->pars: the same values SSS_amg_data_create copies from pars
    SSS_AMG shell;
    std::memset(&shell, 0, sizeof(shell));
    shell.pars = *pars;
    if (!hb_begin(P.b, &shell, o, 0, nullptr)) {
        if (P.b.h) hier_release(P.b.h);
        SSS_amg_setup(mg, A, pars);
        return nullptr;
    }
    P.b.mg = mg;
    (void)hipGetDevice(&P.device);
    std::thread th([&] { P.worker(); });
    sss_amg_setup_hooked(mg, A, pars, pipeline_hook, &P);
    P.t_setup_end = PhaseTimer::now();
    {   // (a setup that returned without its final hook, e.g. no coarse level at all)
        std::lock_guard<std::mutex> lk(P.mu);
        P.finished = true;
    }
    P.cv.notify_all();
    {   // the setup has returned: this thread and the helpers take the remaining level tasks
        const int nh = 2;
        std::vector<std::thread> helpers;
        for (int k = 0; k < nh; ++k)
            helpers.emplace_back([&] {
                (void)hipSetDevice(P.device);
                P.loop(false);
            });
        P.loop(false);
        for (auto &t : helpers) t.join();
    }
    th.join();
    const double t_join = PhaseTimer::now();
    P.b.h->nl = mg->num_levels;
    P.b.h->pars = mg->pars;
    sss_hip_hier *h = pipeline_finish(P, mg);
    if (times) {
        times[0] = P.t_setup_end - t0;                 // setup (with the overlapped uploads)
        times[1] = PhaseTimer::now() - P.t_setup_end;  // mirror work left after the setup returned
        times[2] = t_join - P.t_setup_end;             // of which: waiting for the worker
    }
    return h;
}

// The mirror of a hierarchy already set up: its level tasks (relabel + A_l + smoother plan, P_l /
// R_l) are independent once their inputs exist, so the calling thread and five helpers take them
// side by side (the parity mirror at 7-pt 400^3 took 18.8 s with the tasks in sequence, its largest
// task ~2 s; 3.6 s with three helpers, 3.0 s with five -- profiles/r05_lean_formats/).  A distributed
// engine's replicated tail (level_base > 0) keeps the sequence.
sss_hip_hier *sss::hier_create_impl(const SSS_AMG *mg, const sss_hip_opts *o, int level_base, hipStream_t stream)
{
    Pipeline P;
    HierBuild &b = P.b;
    if (!hb_begin(b, mg, o, level_base, stream)) {
        if (b.h) hier_release(b.h);
        if (b.err) fprintf(stderr, "### ERROR: sss_hip_hier_create: %s\n", b.err.load());
        return nullptr;
    }
    const int nl = mg->num_levels;
    b.h->nl = nl;
    if (level_base != 0 || nl < 3) {
        for (int l = 0; l + 1 < nl; ++l) hb_perm(b, l);
        for (int l = 0; l < nl && !b.err; ++l)
            if (hb_level_a(b, l, l + 1 == nl) && l + 1 < nl) hb_level_pr(b, l);
        return hb_finish(b);
    }
    P.done = nl - 1;   // every level but the coarsest is final
    P.finished = true;
    (void)hipGetDevice(&P.device);
    std::vector<std::thread> helpers;
    for (int k = 0; k < 5; ++k)
        helpers.emplace_back([&] {
            (void)hipSetDevice(P.device);
            P.loop(false);
        });
    P.loop(false);
    for (auto &t : helpers) t.join();
    return pipeline_finish(P, mg);
}

extern "C" sss_hip_hier *sss_hip_hier_create(const SSS_AMG *mg, const sss_hip_opts *o)
{
    return sss::hier_create_impl(mg, o, 0, nullptr);
}

extern "C" void sss_hip_hier_destroy(sss_hip_hier *h) { hier_release(h); }

double *sss::hier_vec(sss_hip_hier *h, int level, int which)
{
    if (!h || level < 0 || level >= h->nl) return nullptr;
    auto &L = h->L[level];
    return which == SSS_HIP_VEC_B ? L.b : which == SSS_HIP_VEC_X ? L.x : which == SSS_HIP_VEC_WP ? L.wp : nullptr;
}

const std::vector<int> &sss::hier_perm(sss_hip_hier *h, int level) { return h->L[level].perm; }

static double *level_vec(sss_hip_hier *h, int level, int which)
{
    if (!h || level < 0 || level >= h->nl) return nullptr;
    auto &L = h->L[level];
    return which == SSS_HIP_VEC_B ? L.b : which == SSS_HIP_VEC_X ? L.x : which == SSS_HIP_VEC_WP ? L.wp : nullptr;
}

extern "C" int sss_hip_upload_vec(sss_hip_hier *h, int level, int which, const double *src, int n)
{
    double *d = level_vec(h, level, which);
    if (!d || n < 0 || n > h->L[level].A.n) return ERROR_INPUT_PAR;
    h->resid_c_ready = false;
    h->pending_f = false;
    const auto &perm = h->L[level].perm;
    if (!perm.empty()) {
        if (n != h->L[level].A.n) return ERROR_INPUT_PAR;   // relabeled levels move whole vectors
        h->stage.resize((size_t)n);
        double *st = h->stage.data();
        parallel_chunks(n, 1 << 16, [&](int lo, int hi) {
            for (int i = lo; i < hi; ++i) st[i] = src[perm[i]];
        });
        src = st;
    }
    SSS_HIP(hipMemcpyAsync(d, src, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, h->stream));
    SSS_HIP(hipStreamSynchronize(h->stream));
    return 0;
}

extern "C" int sss_hip_download_vec(sss_hip_hier *h, int level, int which, double *dst, int n)
{
    double *d = level_vec(h, level, which);
    if (!d || n < 0 || n > h->L[level].A.n) return ERROR_INPUT_PAR;
    if (int rc = hier_stall_check(h)) return rc;   // a stalled pass leaves an invalid iterate
    const auto &perm = h->L[level].perm;
    if (perm.empty()) {
        SSS_HIP(hipMemcpyAsync(dst, d, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, h->stream));
        SSS_HIP(hipStreamSynchronize(h->stream));
        return 0;
    }
    if (n != h->L[level].A.n) return ERROR_INPUT_PAR;
    h->stage.resize((size_t)n);
    double *st = h->stage.data();
    SSS_HIP(hipMemcpyAsync(st, d, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, h->stream));
    SSS_HIP(hipStreamSynchronize(h->stream));
    parallel_chunks(n, 1 << 16, [&](int lo, int hi) {
        for (int i = lo; i < hi; ++i) dst[perm[i]] = st[i];
    });
    return 0;
}

static int coarse_tol(const sss_hip_hier *h, double *tol)
{
    *tol = h->pars.ctol;
    if (*tol > h->pars.tol) *tol = h->pars.tol * 0.1;
    return 0;
}

extern "C" int sss_hip_coarse_solve(sss_hip_hier *h)
{
    auto &C = h->L[h->nl - 1];
    double tol;
    coarse_tol(h, &tol);
    if (h->coarse_mode == SSS_HIP_COARSE_DIRECT) return coarse_direct_apply(h->direct, C.b, C.x, h->stream);
    return coarse_krylov_solve(h->krylov, C.A, C.b, C.x, tol, h->stream);
}

extern "C" int sss_hip_smooth(sss_hip_hier *h, int level, int post)
{
    auto &L = h->L[level];
    const int sweeps = post ? h->pars.post_iter : h->pars.pre_iter;
    h->resid_c_ready = false;
    h->pending_f = false;
    return smoother_run(L.sm, L.A, L.b, L.x, sweeps, h->stream, nullptr, nullptr, nullptr, false, post != 0);
}

// Smoothing that leaves r = b - A x in wp: fused into the last C pass where the plan allows,
// then the F rows by a residual SpMV over blocks [0, split_blk); otherwise a full residual SpMV.
// `partial` (optional): per-block sums of squares of r, for the norm.
static int smooth_then_residual(sss_hip_hier *h, int l, int post, double *partial, const double *pre_f = nullptr,
                                bool x_zero = false)
{
    auto &L = h->L[l];
    const int sweeps = post ? h->pars.post_iter : h->pars.pre_iter;
    ResidFuse rf;
    rf.r = L.wp;
    rf.partial = partial;
    int rc = smoother_run(L.sm, L.A, L.b, L.x, sweeps, h->stream, nullptr, &rf, pre_f, x_zero, post != 0);
    if (rc) return rc;
    if (rf.done) return launch_spmv_blocks(L.A, L.A.split_blk, SSS_HIP_SPMV_RESID, -1.0, L.x, L.b, L.wp, partial, h->stream);
    return launch_spmv(L.A, SSS_HIP_SPMV_RESID, -1.0, L.x, L.b, L.wp, 0, partial, h->stream);
}

// Walks SSS_amg_cycle's static control flow, enqueueing kernels; `coarse(h)` is called where
// the coarsest solve goes.
template <class CoarseFn>
static int walk_cycle(sss_hip_hier *h, CoarseFn coarse, bool pend = false)
{
    const int nl = h->nl;
    const int cycle_type = h->pars.cycle_type <= 0 ? 1 : h->pars.cycle_type;
    int visits[kMaxLevels] = {0};
    int l = 0, rc;
    hipStream_t s = h->stream;
    // per-level timing (sss_hip_time_levels): an event at the end of each step, tagged with its level
    auto mark = [&](int level) -> int {
        if (h->lev_ev.empty() || h->lev_n >= (int)h->lev_ev.size()) return 0;
        h->lev_tag[(size_t)h->lev_n] = level;
        SSS_HIP(hipEventRecord(h->lev_ev[(size_t)h->lev_n++], s));
        return 0;
    };
    if ((rc = mark(-1))) return rc;
    // x_l is zero only on arrival by the descent (restricted into, then cleared): a W-cycle's level
    // re-descended after its post-smoother starts its pre-smoother from that iterate
    bool zeroed = false;
    for (;;) {
        while (l < nl - 1) {
            if (g_ledger) g_ledger->slot = l;
            if (h->tail.from > 0 && l == h->tail.from && cycle_type == 1) {
                // levels tail.from .. nl-1: descent, coarsest solve and ascent in one launch
                {
                    TraceRange tr("levels %d-%d tail", l, nl - 1);
                    if ((rc = tail_launch(h->tail, s))) return rc;
                }
                if ((rc = mark(l))) return rc;
                goto ascent;
            }
            TraceRange tr("level %d descent", l);
            auto &L = h->L[l];
            visits[l]++;
            const bool first = l == 0 && visits[0] == 1;
            // levels >= 1 just zeroed by the descent: the first pass may skip its products
            if ((rc = smooth_then_residual(h, l, 0, nullptr, pend && first ? h->pend_f : nullptr, zeroed && l > 0)))
                return rc;
            if ((rc = launch_spmv(L.R, SSS_HIP_SPMV_MXY, 1.0, L.wp, nullptr, h->L[l + 1].b, 0, nullptr, s))) return rc;
            l++;
            ledger_add(8.0 * h->L[l].A.n);
            SSS_HIP(hipMemsetAsync(h->L[l].x, 0, sizeof(double) * (size_t)h->L[l].A.n, s));
            zeroed = true;
            if ((rc = mark(l - 1))) return rc;
        }
        if (g_ledger) g_ledger->slot = kMaxLevels + 1;
        {
            TraceRange tr("coarse solve (level %d)", nl - 1);
            rc = coarse(h);
        }
        if (rc || (rc = mark(nl - 1))) return rc;
    ascent:
        while (l > 0) {
            l--;
            if (g_ledger) g_ledger->slot = l;
            TraceRange tr("level %d ascent", l);
            auto &L = h->L[l];
            // x_l += P e.  When the post-smoother's first pass overwrites every F row from C values
            // only (depth-1 GS F pass, all |d| > 1e-20), the F rows' correction is dead: prolong
            // into the C rows only (the iterates are bitwise unchanged).
            if (L.sm.f_overwritten && h->pars.post_iter > 0 && L.P.split_row == L.sm.pass[0].hi &&
                L.P.split_row > 0 && L.pinj) {
                if ((rc = launch_prolong_inject(L.P.n - L.P.split_row, L.P.split_row, L.pinj, h->L[l + 1].x, L.x, s)))
                    return rc;
            } else if (L.sm.f_overwritten && h->pars.post_iter > 0 && L.P.split_row == L.sm.pass[0].hi &&
                L.P.split_row > 0 && !L.P.wave_rows && !L.P.vec_rows) {
                if ((rc = launch_spmv_range(L.P, L.P.split_blk, L.P.nblk, SSS_HIP_SPMV_AMXPY, 1.0, h->L[l + 1].x, nullptr,
                                            L.x, nullptr, s)))
                    return rc;
            } else if ((rc = launch_spmv(L.P, SSS_HIP_SPMV_AMXPY, 1.0, h->L[l + 1].x, nullptr, L.x, 0, nullptr, s))) {
                return rc;
            }
            if (l == 0 && L.sm.fuse_resid) {   // the C rows of the outer residual come with the last pass
                ResidFuse rf;
                rf.r = L.wp;
                rf.partial = h->partial;
                if ((rc = smoother_run(L.sm, L.A, L.b, L.x, h->pars.post_iter, s, nullptr, &rf, nullptr, false, true)))
                    return rc;
            } else if ((rc = sss_hip_smooth(h, l, 1))) {
                return rc;
            }
            if ((rc = mark(l))) return rc;
            if (visits[l] < cycle_type) break;
            visits[l] = 0;
        }
        if (l <= 0) break;
        zeroed = false;   // re-descending from level l: x_l holds its post-smoothed iterate
    }
    return 0;
}

// kernel nodes of a captured graph (the cycle's launch count, reported by bench.py)
static int kernel_nodes(hipGraph_t g)
{
    size_t n = 0;
    if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess || n == 0) return 0;
    std::vector<hipGraphNode_t> nodes(n);
    if (hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess) return 0;
    int k = 0;
    for (size_t i = 0; i < n; ++i) {
        hipGraphNodeType t;
        if (hipGraphNodeGetType(nodes[i], &t) == hipSuccess && t == hipGraphNodeTypeKernel) ++k;
    }
    return k;
}

static int end_capture(sss_hip_hier *h, hipGraphExec_t *exec, int *kernels = nullptr)
{
    hipGraph_t g = nullptr;
    SSS_HIP(hipStreamEndCapture(h->stream, &g));
    if (kernels) *kernels += kernel_nodes(g);
    hipError_t e = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    SSS_HIP(e);
    return 0;
}

static int build_cycle_graph(sss_hip_hier *h, bool pend)
{
    std::vector<hipGraphExec_t> &steps = pend ? h->cycle_steps_p : h->cycle_steps;
    int &kern = pend ? h->cycle_kernels_p : h->cycle_kernels;
    kern = 0;
    SSS_HIP(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    int rc = walk_cycle(h, [&steps, &kern](sss_hip_hier *hh) -> int {
        if (hh->coarse_mode == SSS_HIP_COARSE_DIRECT) return sss_hip_coarse_solve(hh);
        hipGraphExec_t seg = nullptr;
        int r = end_capture(hh, &seg, &kern);
        if (r) return r;
        steps.push_back(seg);
        steps.push_back(nullptr);
        SSS_HIP(hipStreamBeginCapture(hh->stream, hipStreamCaptureModeThreadLocal));
        return 0;
    }, pend);
    hipGraphExec_t last = nullptr;
    int rc2 = end_capture(h, &last, &kern);
    if (rc) return rc;
    if (rc2) return rc2;
    steps.push_back(last);
    (pend ? h->cycle_graph_ready_p : h->cycle_graph_ready) = true;
    return 0;
}

static int cycle_impl(sss_hip_hier *h, bool pend);
extern "C" int sss_hip_cycle(sss_hip_hier *h)
{
    const bool pend = h->pending_f && h->nl > 1 && h->pars.pre_iter > 0;
    h->resid_c_ready = false;
    h->pending_f = false;
    int rc = cycle_impl(h, pend);
    if (rc) return rc;
    h->resid_c_ready = h->nl > 1 && h->L[0].sm.fuse_resid && h->pars.post_iter > 0;
    return 0;
}

static int cycle_impl(sss_hip_hier *h, bool pend)
{
    if (!h->opts.use_graph) return walk_cycle(h, [](sss_hip_hier *hh) { return sss_hip_coarse_solve(hh); }, pend);
    if (!(pend ? h->cycle_graph_ready_p : h->cycle_graph_ready)) {
        int rc = build_cycle_graph(h, pend);
        if (rc) return rc;
    }
    for (hipGraphExec_t g : (pend ? h->cycle_steps_p : h->cycle_steps)) {
        if (g) SSS_HIP(hipGraphLaunch(g, h->stream));
        else {
            int rc = sss_hip_coarse_solve(h);
            if (rc) return rc;
        }
    }
    return 0;
}

// f_only: the C rows' residual and partials are already in place (resid_c_ready)
static int enqueue_residual_norm(sss_hip_hier *h, bool f_only)
{
    auto &L = h->L[0];
    const bool pend = f_only && h->pend_f;   // the F half also precomputes the next first F pass
    int rc = pend     ? launch_f_residual_pending(L.sm, L.A, L.b, L.x, L.wp, h->partial, h->pend_f, h->stream)
             : f_only ? launch_spmv_blocks(L.A, L.A.split_blk, SSS_HIP_SPMV_RESID, -1.0, L.x, L.b, L.wp, h->partial,
                                           h->stream)
                      : launch_spmv(L.A, SSS_HIP_SPMV_RESID, -1.0, L.x, L.b, L.wp, 0, h->partial, h->stream);
    if (rc) return rc;
    if ((rc = launch_final_sum(h->partial, L.A.ngrid, h->d_norm, true, h->stream))) return rc;
    return launch_err_flag(h->d_err, h->d_norm + 1, h->stream);
}

// A one-launch GS pass gave up waiting (sss_gs_persist.hip): its iterate is garbage.  Fatal for
// the solve, like the reference's error exits (SSS_utils.c:16-94); the word was cleared on read.
static int stall_error(const char *where)
{
    fprintf(stderr, "### ERROR: %s: an exact Gauss-Seidel pass stalled on the GPU (spin limit reached); "
                    "the iterate is invalid\n", where);
    return ERROR_MISC;
}

int sss::hier_stall_check(sss_hip_hier *h)
{
    if (!h || !h->d_err) return 0;
    if (int rc = launch_err_flag(h->d_err, h->d_norm + 1, h->stream)) return rc;
    SSS_HIP(hipMemcpyAsync(h->h_norm + 1, h->d_norm + 1, sizeof(double), hipMemcpyDeviceToHost, h->stream));
    SSS_HIP(hipStreamSynchronize(h->stream));
    return h->h_norm[1] != 0.0 ? stall_error("sss_hip engine") : 0;
}

unsigned *sss::hier_err_word(sss_hip_hier *h) { return h ? h->d_err : nullptr; }
bool sss::hier_coarse_on_device(sss_hip_hier *h) { return h && h->coarse_mode == SSS_HIP_COARSE_DIRECT; }
void sss::hier_set_err_word(sss_hip_hier *h, unsigned *err)
{
    for (int l = 0; l + 1 < h->nl; ++l) smoother_set_err(h->L[l].sm, err);
}

extern "C" int sss_hip_residual_norm(sss_hip_hier *h, double *absres)
{
    const bool f_only = h->resid_c_ready;
    if (h->opts.use_graph) {
        hipGraphExec_t &exec = f_only ? h->resid_f_exec : h->resid_exec;
        if (!exec) {
            SSS_HIP(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
            int rc = enqueue_residual_norm(h, f_only);
            hipGraphExec_t ex = nullptr;
            int rc2 = end_capture(h, &ex);
            if (rc) return rc;
            if (rc2) return rc2;
            exec = ex;
        }
        SSS_HIP(hipGraphLaunch(exec, h->stream));
    } else {
        int rc = enqueue_residual_norm(h, f_only);
        if (rc) return rc;
    }
    h->pending_f = f_only && h->pend_f;
    SSS_HIP(hipMemcpyAsync(h->h_norm, h->d_norm, 2 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    SSS_HIP(hipStreamSynchronize(h->stream));
    *absres = h->h_norm[0];
    if (h->h_norm[1] != 0.0) {
        h->pending_f = h->resid_c_ready = false;
        return stall_error("sss_hip_residual_norm");
    }
    return 0;
}

// AMG as a preconditioner (not in the reference, whose CG/GMRES serve only
// the coarsest level): flexible CG with Polak-Ribiere beta, one V-cycle of this hierarchy (its
// configured smoothers and coarse solve) per iteration as M^-1.  Right-hand side L0.b, initial
// guess and result L0.x; iterates until ||r_k|| / ||b|| < tol (recursive residual) or maxit.
// Dots are fixed-order reductions (deterministic); one 8-byte read-back per iteration.
extern "C" int sss_hip_pcg(sss_hip_hier *h, double tol, int maxit, int *iters, double *relres, double *hist,
                           int hist_cap)
{
    auto &L = h->L[0];
    const int n = L.A.n;
    hipStream_t s = h->stream;
    if (!h->pcg_v) {
        h->pcg_v = dev_alloc<double>((size_t)7 * n);
        h->pcg_part = dev_alloc<double>(1024 + kFinalScratch);
        h->pcg_s = dev_alloc<double>(8);
        if (!h->pcg_v || !h->pcg_part || !h->pcg_s) return hip_fail(hipErrorOutOfMemory, "hipMalloc(pcg)", __FILE__, __LINE__);
        SSS_HIP(hipHostMalloc((void **)&h->pcg_h, 8 * sizeof(double), hipHostMallocDefault));
    }
    h->pending_f = false;   // b and x are rewritten below
    double *bs = h->pcg_v, *xs = bs + n, *r = xs + n, *z = r + n, *p = z + n, *q = p + n, *ro = q + n;
    double *rz = h->pcg_s, *pq = h->pcg_s + 1, *rr = h->pcg_s + 2, *rzn = h->pcg_s + 3, *roz = h->pcg_s + 4;
    const size_t bytes = sizeof(double) * (size_t)n;
    int rc;
    auto precondition = [&](const double *rin, double *zout) -> int {   // zout = one V-cycle on (rin, 0)
        SSS_HIP(hipMemcpyAsync(L.b, rin, bytes, hipMemcpyDeviceToDevice, s));
        SSS_HIP(hipMemsetAsync(L.x, 0, bytes, s));
        int c = sss_hip_cycle(h);
        if (c) return c;
        SSS_HIP(hipMemcpyAsync(zout, L.x, bytes, hipMemcpyDeviceToDevice, s));
        return 0;
    };
    auto fetch = [&](const double *dv, double *out) -> int {
        SSS_HIP(hipMemcpyAsync(h->pcg_h, dv, sizeof(double), hipMemcpyDeviceToHost, s));
        SSS_HIP(hipStreamSynchronize(s));
        *out = h->pcg_h[0];
        return 0;
    };
    SSS_HIP(hipMemcpyAsync(bs, L.b, bytes, hipMemcpyDeviceToDevice, s));
    SSS_HIP(hipMemcpyAsync(xs, L.x, bytes, hipMemcpyDeviceToDevice, s));
    double nb2 = 0.0, rr_h = 0.0, rel = 1.0;
    if ((rc = launch_dot(n, bs, bs, h->pcg_part, rr, s)) || (rc = fetch(rr, &nb2))) return rc;
    const double nb = std::sqrt(nb2);
    int it = 0;
    if (nb == 0.0) {
        SSS_HIP(hipMemsetAsync(L.x, 0, bytes, s));
    } else {
        if ((rc = launch_spmv(L.A, SSS_HIP_SPMV_RESID, -1.0, xs, bs, r, 0, nullptr, s))) return rc;   // r = b - A x
        if ((rc = precondition(r, z))) return rc;
        if ((rc = launch_dot(n, r, z, h->pcg_part, rz, s))) return rc;
        SSS_HIP(hipMemcpyAsync(p, z, bytes, hipMemcpyDeviceToDevice, s));
        while (it < maxit) {
            ++it;
            if ((rc = launch_spmv(L.A, SSS_HIP_SPMV_MXY, 1.0, p, nullptr, q, 0, nullptr, s))) return rc;   // q = A p
            if ((rc = launch_dot(n, p, q, h->pcg_part, pq, s))) return rc;
            if ((rc = launch_axpy_ratio(n, rz, pq, 1.0, p, xs, s))) return rc;                          // x += a p
            SSS_HIP(hipMemcpyAsync(ro, r, bytes, hipMemcpyDeviceToDevice, s));
            if ((rc = launch_axpy_ratio(n, rz, pq, -1.0, q, r, s))) return rc;                          // r -= a q
            if ((rc = launch_dot(n, r, r, h->pcg_part, rr, s)) || (rc = fetch(rr, &rr_h))) return rc;
            rel = std::sqrt(rr_h) / nb;
            if (hist && it <= hist_cap) hist[it - 1] = rel;
            if (rel < tol) break;
            if ((rc = precondition(r, z))) return rc;
            if ((rc = launch_dot(n, r, z, h->pcg_part, rzn, s))) return rc;
            if ((rc = launch_dot(n, ro, z, h->pcg_part, roz, s))) return rc;
            if ((rc = launch_xpby_ratio(n, rzn, roz, rz, z, p, s))) return rc;   // p = z + ((r-ro).z / rz) p
            SSS_HIP(hipMemcpyAsync(rz, rzn, sizeof(double), hipMemcpyDeviceToDevice, s));
        }
        SSS_HIP(hipMemcpyAsync(L.x, xs, bytes, hipMemcpyDeviceToDevice, s));
    }
    SSS_HIP(hipMemcpyAsync(L.b, bs, bytes, hipMemcpyDeviceToDevice, s));
    SSS_HIP(hipStreamSynchronize(s));
    h->resid_c_ready = false;
    if (iters) *iters = it;
    if (relres) *relres = rel;
    return hier_stall_check(h);
}

extern "C" int sss_hip_sync(sss_hip_hier *h)
{
    SSS_HIP(hipStreamSynchronize(h->stream));
    return hier_stall_check(h);
}

extern "C" int sss_hip_num_levels(sss_hip_hier *h) { return h ? h->nl : 0; }

// The stored-format bytes one outer iteration's kernels read and write (sss_engine.hpp ByteLedger):
// the cycle as sss_hip_cycle would run it next, and the residual + norm after it, walked into a
// stream capture that is discarded (nothing executes).  out[l] for level l < nslots - 2 (coarse
// levels of a single-workgroup tail land on its first level), out[nslots - 2] the outer residual +
// norm, out[nslots - 1] the coarsest solve (explicit inverse; the device Krylov solver is not
// counted).  nslots >= num_levels + 2.
extern "C" int sss_hip_cycle_bytes(sss_hip_hier *h, double *out, int nslots)
{
    if (!h || !out || nslots < h->nl + 2) return ERROR_INPUT_PAR;
    const bool pend = h->pending_f && h->nl > 1 && h->pars.pre_iter > 0;
    const bool f_only_next = h->nl > 1 && h->L[0].sm.fuse_resid && h->pars.post_iter > 0;
    const bool keep_pending = h->pending_f, keep_ready = h->resid_c_ready;
    ByteLedger led;
    SSS_HIP(hipStreamSynchronize(h->stream));
    SSS_HIP(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    g_ledger = &led;
    int rc = walk_cycle(h, [](sss_hip_hier *hh) {
        return hh->coarse_mode == SSS_HIP_COARSE_DIRECT ? coarse_direct_apply(hh->direct, hh->L[hh->nl - 1].b,
                                                                              hh->L[hh->nl - 1].x, hh->stream)
                                                        : 0;
    }, pend);
    led.slot = kMaxLevels;
    if (!rc) rc = enqueue_residual_norm(h, f_only_next);
    g_ledger = nullptr;
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(h->stream, &g);
    if (g) (void)hipGraphDestroy(g);
    h->pending_f = keep_pending;
    h->resid_c_ready = keep_ready;
    if (rc) return rc;
    SSS_HIP(e);
    for (int i = 0; i < nslots; ++i) out[i] = 0.0;
    for (int l = 0; l < h->nl && l < kMaxLevels; ++l) out[l] = led.bytes[l];
    out[nslots - 2] = led.bytes[kMaxLevels];
    out[nslots - 1] = led.bytes[kMaxLevels + 1];
    return 0;
}

extern "C" int sss_hip_tail_from(sss_hip_hier *h) { return h ? h->tail.from : -1; }

extern "C" int sss_hip_cycle_launches(sss_hip_hier *h)
{
    if (!h || !(h->cycle_graph_ready || h->cycle_graph_ready_p)) return -1;
    return h->cycle_graph_ready_p ? h->cycle_kernels_p : h->cycle_kernels;
}

extern "C" int sss_hip_level_info_get(sss_hip_hier *h, int level, sss_hip_level_info *out)
{
    if (!h || level < 0 || level >= h->nl) return ERROR_INPUT_PAR;
    auto &L = h->L[level];
    out->rows = L.A.n;
    out->nnz = L.A.nnz;
    out->nnz_p = L.P.nnz;
    out->dag_f = L.sm.pass[0].depth;
    out->dag_c = L.sm.pass[1].depth;
    out->smoother_kind = L.sm.kind;
    out->inner = L.sm.inner;
    out->gs_engine_f = L.sm.fz.engine ? 3 : L.sm.pass[0].gp.engine;   // 3: all passes in one launch
    out->gs_engine_c = L.sm.fz.engine ? 3 : L.sm.pass[1].gp.engine;
    unsigned ef = 0, ec = 0, ez = 0;
    if (gs_persist_error(L.sm.pass[0], &ef) || gs_persist_error(L.sm.pass[1], &ec)) return ERROR_MISC;
    if (L.sm.fz.err && hipMemcpy(&ez, L.sm.fz.err, sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess)
        return ERROR_MISC;
    out->gs_stall = (int)(ef | ec | ez);
    auto fmt = [](const DevCSR &M) {
        return (M.pk ? 1 : 0) | (has_dict(M) ? 2 : 0) | (M.vec_rows ? 4 : 0) | (M.mg_G ? 8 : 0) | (M.wave_rows ? 16 : 0) |
               (M.dv_ell ? 64 : 0) | (M.dv_xell ? 128 : 0);
    };
    out->a_format = fmt(L.A);
    out->r_format = level + 1 < h->nl ? fmt(L.R) : 0;
    out->p_format = level + 1 < h->nl ? fmt(L.P) : 0;
    out->a_stream_bytes = L.A.stream_bytes;
    return 0;
}

// Per-level time of the cycle: level_ms[l] = level l's steps (pre-smoothing, residual, restriction,
// zero fill; prolongation, post-smoothing; the coarsest level: its solve; a single-workgroup tail:
// at its first level), averaged over reps eager cycles with an event between the steps (launch gaps
// included, unlike the graph-replayed cycle).  Advances the iterate.  nslots >= num levels.
extern "C" int sss_hip_time_levels(sss_hip_hier *h, int reps, double *level_ms, int nslots)
{
    if (!h || reps < 1 || nslots < h->nl) return ERROR_INPUT_PAR;
    const size_t nev = (size_t)4 * h->nl + 4;
    h->lev_ev.assign(nev, nullptr);
    h->lev_tag.assign(nev, -1);
    int rc = 0;
    for (auto &e : h->lev_ev)
        if (hipEventCreate(&e) != hipSuccess) rc = ERROR_MISC;
    std::vector<double> acc((size_t)h->nl, 0.0);
    for (int r = 0; r < reps && !rc; ++r) {
        h->lev_n = 0;
        h->resid_c_ready = h->pending_f = false;
        rc = walk_cycle(h, [](sss_hip_hier *hh) { return sss_hip_coarse_solve(hh); }, false);
        if (!rc && hipStreamSynchronize(h->stream) != hipSuccess) rc = ERROR_MISC;
        for (int k = 1; k < h->lev_n && !rc; ++k) {
            float t = 0.0f;
            if (hipEventElapsedTime(&t, h->lev_ev[(size_t)k - 1], h->lev_ev[(size_t)k]) != hipSuccess) rc = ERROR_MISC;
            const int lv = h->lev_tag[(size_t)k];
            if (lv >= 0 && lv < h->nl) acc[(size_t)lv] += t;
        }
    }
    for (hipEvent_t e : h->lev_ev)
        if (e) (void)hipEventDestroy(e);
    h->lev_ev.clear();
    h->lev_tag.clear();
    h->lev_n = 0;
    h->resid_c_ready = h->pending_f = false;
    if (rc) return rc;
    for (int l = 0; l < h->nl; ++l) level_ms[l] = acc[(size_t)l] / reps;
    return 0;
}

extern "C" int sss_hip_time_level0_spmv(sss_hip_hier *h, int reps, double *avg_ms)
{
    auto &L = h->L[0];
    SSS_HIP(hipStreamSynchronize(h->stream));
    SSS_HIP(hipEventRecord(h->ev0, h->stream));
    for (int r = 0; r < reps; ++r) {
        int rc = launch_spmv(L.A, SSS_HIP_SPMV_RESID, -1.0, L.x, L.b, L.wp, 0, nullptr, h->stream);
        if (rc) return rc;
    }
    SSS_HIP(hipEventRecord(h->ev1, h->stream));
    SSS_HIP(hipEventSynchronize(h->ev1));
    float ms = 0.f;
    SSS_HIP(hipEventElapsedTime(&ms, h->ev0, h->ev1));
    *avg_ms = (double)ms / reps;
    return 0;
}

// The same residual SpMV of level 0 from its plain CSR arrays (row_ptr, col_idx, val; always
// resident), whatever storage the cycle uses: the fine-level CSR SpMV of the metric.
extern "C" int sss_hip_time_level0_spmv_csr(sss_hip_hier *h, int reps, double *avg_ms)
{
    auto &L = h->L[0];
    // (column ELL blocks are not tile-sized: the stored format is timed instead)
    if (L.A.wave_rows || L.A.vec_rows || L.A.dv_xell) return sss_hip_time_level0_spmv(h, reps, avg_ms);
    DevCSR c = L.A;   // a view: the CSR arrays and row blocks only (never freed through c)
    c.pk = nullptr;
    c.pv = nullptr;
    c.pb = nullptr;
    c.dv_ell = nullptr;
    c.dv_code = nullptr;
    c.dv_vi = nullptr;
    SSS_HIP(hipStreamSynchronize(h->stream));
    SSS_HIP(hipEventRecord(h->ev0, h->stream));
    for (int r = 0; r < reps; ++r) {
        int rc = launch_spmv(c, SSS_HIP_SPMV_RESID, -1.0, L.x, L.b, L.wp, 0, nullptr, h->stream);
        if (rc) return rc;
    }
    SSS_HIP(hipEventRecord(h->ev1, h->stream));
    SSS_HIP(hipEventSynchronize(h->ev1));
    float ms = 0.f;
    SSS_HIP(hipEventElapsedTime(&ms, h->ev0, h->ev1));
    *avg_ms = (double)ms / reps;
    return 0;
}

extern "C" int sss_hip_time_iterations(sss_hip_hier *h, int reps, double *avg_ms, double *absres)
{
    SSS_HIP(hipStreamSynchronize(h->stream));
    SSS_HIP(hipEventRecord(h->ev0, h->stream));
    for (int r = 0; r < reps; ++r) {
        int rc = sss_hip_cycle(h);
        if (!rc) rc = sss_hip_residual_norm(h, absres);
        if (rc) return rc;
    }
    SSS_HIP(hipEventRecord(h->ev1, h->stream));
    SSS_HIP(hipEventSynchronize(h->ev1));
    float ms = 0.f;
    SSS_HIP(hipEventElapsedTime(&ms, h->ev0, h->ev1));
    *avg_ms = (double)ms / reps;
    return 0;
}

// ---- host-memory convenience wrappers for the exported reference entry points ----------------
// The reference's spmv_cuda re-copies the whole CSR on every call (Solve/SSS_cuda.cu:124-139).
// Here the device form of a matrix (and of a smoother plan / coarse solver built on it) is kept in
// a small cache keyed by the matrix contents: a content hash of row_ptr / col_idx / val (host
// memory, row-parallel; far cheaper than the upload and the format build) plus the dimensions and
// the use.  A caller that loops over these entry points with the same operator pays the upload
// once; a caller that changes the matrix in place gets a fresh upload (the hash changes).
// sss_hip_host_cache_clear() releases everything.  The smoother and coarse-solver objects hold
// mutable device state (the one-launch GS engine's tickets and granules, the Krylov scratch), so
// each call holds its entry's mutex for the whole apply; operators above SSS_HIP_HOST_CACHE_MB
// (default 1024 MiB of CSR) are built for the call and released after it, not cached.
extern char **environ;

namespace {
struct HostCSR {
    DevCSR d;
    ~HostCSR() { devcsr_free(d); }
};
struct HostSmooth {
    std::mutex run;   // held for a whole apply (shared mutable device state)
    DevCSR d;
    SmootherPlan sp;
    ~HostSmooth()
    {
        smoother_free(sp);
        devcsr_free(d);
    }
};
struct HostCoarse {
    std::mutex run;   // held for a whole apply (Krylov scratch)
    DevCSR d;
    CoarseDirect cd;
    bool direct = false;
    CoarseKrylov *k = nullptr;
    ~HostCoarse()
    {
        if (direct) coarse_direct_free(cd);
        coarse_krylov_destroy(k);
        devcsr_free(d);
    }
};

inline unsigned long long mix64(unsigned long long h, unsigned long long w)
{
    h ^= w * 0x9E3779B97F4A7C15ull;
    h = (h << 31) | (h >> 33);
    return h * 0xC2B2AE3D27D4EB4Full;
}
// content hash of n bytes: fixed chunks hashed in parallel, combined in chunk order
unsigned long long hash_bytes(const void *p, size_t n, unsigned long long seed)
{
    const unsigned char *b = static_cast<const unsigned char *>(p);
    constexpr size_t kChunk = (size_t)1 << 20;
    const int nc = (int)((n + kChunk - 1) / kChunk);
    std::vector<unsigned long long> part((size_t)std::max(nc, 1), 0);
    parallel_chunks(nc, 1, [&](int c0, int c1) {
        for (int c = c0; c < c1; ++c) {
            const size_t lo = (size_t)c * kChunk, hi = std::min(n, lo + kChunk);
            unsigned long long h = 0x2545F4914F6CDD1Dull ^ (unsigned long long)c;
            size_t i = lo;
            for (; i + 8 <= hi; i += 8) {
                unsigned long long w;
                std::memcpy(&w, b + i, 8);
                h = mix64(h, w);
            }
            for (; i < hi; ++i) h = mix64(h, b[i]);
            part[(size_t)c] = h;
        }
    });
    unsigned long long h = mix64(seed, n);
    for (auto v : part) h = mix64(h, v);
    return h;
}
unsigned long long matrix_key(const SSS_MAT &A, unsigned long long use)
{
    int dev = 0;
    (void)hipGetDevice(&dev);   // device objects belong to the current device
    unsigned long long h = mix64(mix64(use, (unsigned long long)dev), (unsigned long long)A.num_rows);
    // the upload and plan builders read SSS_HIP_* switches (formats, kernel paths): part of the key
    for (char **e = environ; e && *e; ++e)
        if (std::strncmp(*e, "SSS_HIP_", 8) == 0) h = hash_bytes(*e, std::strlen(*e), h);
    h = mix64(h, (unsigned long long)A.num_cols);
    h = mix64(h, (unsigned long long)A.num_nnzs);
    h = hash_bytes(A.row_ptr, sizeof(int) * ((size_t)A.num_rows + 1), h);
    h = hash_bytes(A.col_idx, sizeof(int) * (size_t)A.num_nnzs, h);
    return hash_bytes(A.val, sizeof(double) * (size_t)A.num_nnzs, h);
}

struct PreparedCache {
    struct Entry {
        unsigned long long key;
        std::shared_ptr<void> obj;
        unsigned long long tick;
    };
    std::mutex mu;
    std::vector<Entry> e;
    unsigned long long tick = 0;
    static constexpr size_t kMax = 4;
    // cache: false builds a private object for this call (operators too large to keep resident)
    template <class T, class Build>
    std::shared_ptr<T> get(unsigned long long key, Build build, bool cache = true)
    {
        if (!cache) return build();
        {
            std::lock_guard<std::mutex> lk(mu);
            for (auto &x : e)
                if (x.key == key) {
                    x.tick = ++tick;
                    return std::static_pointer_cast<T>(x.obj);
                }
        }
        std::shared_ptr<T> obj = build();
        if (!obj) return obj;
        std::lock_guard<std::mutex> lk(mu);
        if (e.size() >= kMax) {
            auto old = std::min_element(e.begin(), e.end(), [](const Entry &a, const Entry &b) { return a.tick < b.tick; });
            e.erase(old);
        }
        e.push_back({key, obj, ++tick});
        return obj;
    }
    void clear()
    {
        std::lock_guard<std::mutex> lk(mu);
        e.clear();
    }
};
bool cacheable(const SSS_MAT &A)
{
    const char *e = getenv("SSS_HIP_HOST_CACHE_MB");
    const double mb = (e && *e) ? atof(e) : 1024.0;
    return 12.0 * (double)A.num_nnzs + 4.0 * (double)A.num_rows <= mb * 1048576.0;
}
PreparedCache &prepared()
{
    static PreparedCache *c = new PreparedCache();   // objects hold device memory: never torn down at exit
    return *c;
}
}  // namespace

extern "C" void sss_hip_host_cache_clear(void) { prepared().clear(); }

extern "C" int sss_hip_host_spmv(int op, double alpha, const SSS_MAT *A, const double *x, const double *b,
                                 double *y, int cap)
{
    if (sss_hip_device_count() <= 0) return ERROR_MISC;
    sss_hip_opts o;
    sss_hip_opts_default(&o);   // SSS_HIP_SORTED_TILES; always the reference's summation order here
    // rectangular operators (P, R) may take the dictionary ELL, as the hierarchy's restrictions
    int enc = level_encoding(o) & (kEncSortedTiles | kEncDict);
    if (A->num_rows != A->num_cols) enc = restriction_encoding(o) & (kEncSortedTiles | kEncEll);
    auto M = prepared().get<HostCSR>(matrix_key(*A, 0x5350ull ^ ((unsigned long long)enc << 8)), [&] {
        auto m = std::make_shared<HostCSR>();
        return devcsr_upload(m->d, *A, -1, enc) ? nullptr : m;
    }, cacheable(*A));
    if (!M) return ERROR_MISC;
    const size_t ny = (size_t)A->num_rows, nx = (size_t)A->num_cols;
    double *dx = dev_alloc<double>(nx), *dy = dev_alloc<double>(ny), *db = dev_alloc<double>(ny);
    int rc = 0;
    if (!dx || !dy || !db) rc = ERROR_ALLOC_MEM;
    if (!rc && hipMemcpy(dx, x, sizeof(double) * nx, hipMemcpyHostToDevice) != hipSuccess) rc = ERROR_MISC;
    if (!rc && hipMemcpy(dy, y, sizeof(double) * ny, hipMemcpyHostToDevice) != hipSuccess) rc = ERROR_MISC;
    if (!rc && b && hipMemcpy(db, b, sizeof(double) * ny, hipMemcpyHostToDevice) != hipSuccess) rc = ERROR_MISC;
    if (!rc) rc = launch_spmv(M->d, op, alpha, dx, db, dy, cap, nullptr, nullptr);
    if (!rc && hipMemcpy(y, dy, sizeof(double) * ny, hipMemcpyDeviceToHost) != hipSuccess) rc = ERROR_MISC;
    dev_free(dx);
    dev_free(dy);
    dev_free(db);
    return rc;
}

extern "C" int sss_hip_host_smooth(const SSS_SMTR *s, int post)
{
    if (sss_hip_device_count() <= 0) return ERROR_MISC;
    const int n = s->A->num_rows;
    const int use_cf = s->cf_order && s->ordering;
    const bool natural = !use_cf && s->smoother == SSS_SM_GS;
    // natural order (Solve/SSS_smooth.c:171-176, 256-260): pre i = istart .. iend, post i = iend ..
    // istart, by istep; a loop whose bounds are crossed for its direction runs no row
    const int i1 = post ? s->iend : s->istart, in = post ? s->istart : s->iend, step = s->istep;
    if (natural && step != 1 && step != -1) {
        fprintf(stderr, "### ERROR: natural-order Gauss-Seidel on the GPU needs istep = +1 or -1 (got %d)\n", step);
        return ERROR_INPUT_PAR;
    }
    const bool desc = step < 0;
    const int lo = desc ? in : i1, hi = (desc ? i1 : in) + 1;
    if (natural && (lo < 0 || hi > n)) return ERROR_INPUT_PAR;
    if (natural && lo >= hi) return 0;
    const int kind = s->smoother == SSS_SM_JACOBI ? SSS_HIP_SMOOTH_JACOBI : SSS_HIP_SMOOTH_EXACT;
    unsigned long long use = mix64(0x534Dull, natural ? 1 : 0);
    use = mix64(use, (unsigned long long)kind);
    if (natural) use = mix64(mix64(use, (unsigned long long)lo), (unsigned long long)hi);
    if (use_cf) use = hash_bytes(s->ordering, sizeof(int) * (size_t)n, use);
    auto M = prepared().get<HostSmooth>(matrix_key(*s->A, use), [&] {
        auto m = std::make_shared<HostSmooth>();
        if (devcsr_upload(m->d, *s->A)) return std::shared_ptr<HostSmooth>();
        if (natural ? smoother_build_natural(m->sp, *s->A, lo, hi)
                    : smoother_build(m->sp, *s->A, use_cf ? s->ordering : nullptr, kind))
            return std::shared_ptr<HostSmooth>();
        return m;
    }, cacheable(*s->A));
    if (!M) return ERROR_MISC;
    std::lock_guard<std::mutex> run_lock(M->run);
    double *dx = dev_alloc<double>((size_t)n), *db = dev_alloc<double>((size_t)n);
    int rc = (!dx || !db) ? ERROR_ALLOC_MEM : 0;
    if (!rc && hipMemcpy(dx, s->x->d, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess) rc = ERROR_MISC;
    if (!rc && hipMemcpy(db, s->b->d, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess) rc = ERROR_MISC;
    // a caller's iterate of +0.0 everywhere (every bit zero) takes the zero-iterate forms the cycle uses
    // on a just-cleared level (the fused engine's reduced sweep-0 rows, the C/F-Jacobi first pass
    // without the matrix): bitwise the full sweep on finite values, with b_i = -0.0 handled
    bool x_zero = !natural;
    for (int i = 0; x_zero && i < n; ++i) {
        unsigned long long u;
        memcpy(&u, s->x->d + i, sizeof u);
        x_zero = u == 0ull;
    }
    if (!rc) rc = smoother_run(M->sp, M->d, db, dx, s->nsweeps, nullptr, nullptr, nullptr, nullptr, x_zero, natural && desc);
    if (!rc && hipMemcpy(s->x->d, dx, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess) rc = ERROR_MISC;
    // a stalled one-launch pass or fused call: fail, and clear its word for the next call (read every
    // word even after a failure, so none stays set)
    bool stalled = false;
    for (auto &ps : M->sp.pass) {
        unsigned e = 0;
        if (gs_persist_error(ps, &e)) rc = rc ? rc : ERROR_MISC;
        if (e) {
            (void)hipMemset(ps.gp.err, 0, sizeof(unsigned));
            stalled = true;
        }
    }
    unsigned ez = 0;
    if (gs_fused_error(M->sp.fz, &ez, true)) rc = rc ? rc : ERROR_MISC;
    if (ez) stalled = true;
    if (stalled && !rc) rc = stall_error("SSS_amg_smoother_pre/post");
    dev_free(dx);
    dev_free(db);
    return rc;
}

extern "C" int sss_hip_host_coarse_solve(SSS_MAT *A, SSS_VEC *b, SSS_VEC *x, double ctol, int coarse_mode,
                                         int row_cap)
{
    if (sss_hip_device_count() <= 0) return ERROR_MISC;
    const int n = A->num_rows;
    const bool direct = coarse_mode == SSS_HIP_COARSE_DIRECT && n <= 20000;
    auto M = prepared().get<HostCoarse>(
        matrix_key(*A, mix64(mix64(0x4353ull, direct ? 1 : 0), (unsigned long long)row_cap)), [&] {
            auto m = std::make_shared<HostCoarse>();
            if (devcsr_upload(m->d, *A)) return std::shared_ptr<HostCoarse>();
            if (direct) {
                if (coarse_direct_build(m->cd, *A, nullptr)) return std::shared_ptr<HostCoarse>();
                m->direct = true;
            } else {
                m->k = coarse_krylov_create(m->d, row_cap, nullptr);
                if (!m->k) return std::shared_ptr<HostCoarse>();
            }
            return m;
        }, cacheable(*A));
    if (!M) return ERROR_MISC;
    std::lock_guard<std::mutex> run_lock(M->run);
    double *dx = dev_alloc<double>((size_t)n), *db = dev_alloc<double>((size_t)n);
    int rc = (!dx || !db) ? ERROR_ALLOC_MEM : 0;
    if (!rc && hipMemcpy(dx, x->d, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess) rc = ERROR_MISC;
    if (!rc && hipMemcpy(db, b->d, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess) rc = ERROR_MISC;
    if (!rc) {
        if (direct) {
            rc = coarse_direct_apply(M->cd, db, dx, nullptr);
            if (!rc && hipDeviceSynchronize() != hipSuccess) rc = ERROR_MISC;
        } else {
            rc = coarse_krylov_solve(M->k, M->d, db, dx, ctol, nullptr);
        }
    }
    if (!rc && hipMemcpy(x->d, dx, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess) rc = ERROR_MISC;
    dev_free(dx);
    dev_free(db);
    return rc;
}
