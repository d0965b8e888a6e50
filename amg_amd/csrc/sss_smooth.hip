// sss_smooth.hip — smoothers of the V-cycle (gfx950, fp64, no contraction).
//
// Exact GS-CF (replaces SSS_amg_smoother_gs_cf, Solve/SSS_smooth.c:4-87; dispatched from
// SSS_amg_smoother_pre/post :138-304).  Per sweep the reference runs an F pass (mark != 1,
// ascending rows) then a C pass (mark == 1, ascending rows), updating x in place:
//     t = b_i - sum_{k: j_k != i} a_k * x_{j_k}   (in stored order), x_i = t / d
// where d is the last diagonal entry seen so far in the call (it is stale for a row without a
// diagonal entry).  Inside one pass, row i needs the NEW x_j of same-class rows j < i it is
// coupled to and the OLD x_j of same-class rows j > i.  Level scheduling reproduces exactly
// that: depth(i) = 1 + max depth of coupled same-class rows j < i (read-after-write), and
// every coupled same-class row j > i is pushed below i (write-after-read, for nonsymmetric
// patterns).  Rows of equal depth are independent; each depth is one launch.  The result is
// bitwise identical to the sequential reference (same per-row operation order).
//
// On level 0 of the 7-point Poisson operator the RS split is red-black, so each pass has depth
// 1 — a single fully parallel, HBM-bound launch.  Coarser levels have
// depth in the hundreds; there the passes are launch-latency-bound.
//
// C/F-Jacobi (engine extension; SSS_SM_JACOBI): F pass then C pass, every row of a pass
// reading the values from before the pass (ping-pong buffers), d = the row's last diagonal.
#include "sss_engine.hpp"
#include "sss_spmv_dev.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <type_traits>
#include <cmath>

namespace sss {

// ---- host-side planning ---------------------------------------------------------------------
template <class T>
static int upload_array(T **dst, const T *src, size_t count)
{
    *dst = dev_alloc<T>(count);
    if (!*dst) return hip_fail(hipErrorOutOfMemory, "hipMalloc(plan array)", __FILE__, __LINE__);
    return count == 0 ? 0 : h2d(*dst, src, sizeof(T) * count);
}
static int upload_ints(int **dst, const std::vector<int> &src) { return upload_array(dst, src.data(), src.size()); }
static int upload_ints(int **dst, const HostBuf<int> &src) { return upload_array(dst, src.data(), src.size()); }
static int upload_doubles(double **dst, const HostBuf<double> &src) { return upload_array(dst, src.data(), src.size()); }
static int upload_doubles(double **dst, const std::vector<double> &src) { return upload_array(dst, src.data(), src.size()); }

int smoother_build(SmootherPlan &sp, const SSS_MAT &A, const int *mark, int kind, const DevCSR *dA, int inner,
                   const int *gcls, int enc)
{
    const int n = A.num_rows;
    const int *rp = A.row_ptr, *ci = A.col_idx;
    const double *v = A.val;
    // per-row arrays filled by the row-parallel pass below (no serial zero-fill of n-length arrays)
    HostBuf<int> cls, depth, pushed, diag_pos;
    HostBuf<double> last_diag, d_first_buf, d_later_buf;
    HostBuf<char> has_diag;
    cls.resize(n), depth.resize(n), pushed.resize(n), diag_pos.resize(n), last_diag.resize(n), has_diag.resize(n);
    bool all_diag = true, single_diag = true;
    int rc;
    const char *tz = getenv("SSS_HIP_TILE_DIAG");   // 0: divisors from the deff stream (tests)

    const bool timing = getenv("SSS_HIP_TIMING") != nullptr;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double t0 = now(), t_sched = 0, t_persist = 0, t_two = 0;
    sp.kind = kind;
    {   // classes, diagonals (row-parallel)
        std::atomic<bool> all{true}, single{true};
        parallel_chunks(n, 1 << 16, [&](int lo, int hi) {
            bool a = true, s1 = true;
            for (int i = lo; i < hi; ++i) {
                cls[i] = mark ? (mark[i] == 1 ? 1 : 0) : 0;
                depth[i] = pushed[i] = 0;
                last_diag[i] = 0.0;
                has_diag[i] = 0;
                diag_pos[i] = -1;
                for (int k = rp[i]; k < rp[i + 1]; ++k)
                    if (ci[k] == i) {
                        last_diag[i] = v[k];
                        if (has_diag[i]) s1 = false;
                        has_diag[i] = 1;
                        diag_pos[i] = k;
                    }
                a = a && has_diag[i];
            }
            if (!a) all = false;
            if (!s1) single = false;
        });
        all_diag = all;
        single_diag = single;
    }
    // stale-d resolution: simulate the divisor register over two sweeps of (F pass, C pass); with
    // a diagonal in every row it is each row's own last diagonal entry
    const double *d_first = last_diag.data(), *d_later = last_diag.data();
    if (!all_diag) {
        d_first_buf.resize(n), d_later_buf.resize(n);
        d_first = d_first_buf.data(), d_later = d_later_buf.data();
        double d = 0.0;
        for (int sweep = 0; sweep < 2; ++sweep)
            for (int c = 0; c < 2; ++c)
                for (int i = 0; i < n; ++i) {
                    if (cls[i] != c) continue;
                    if (has_diag[i]) d = last_diag[i];
                    (sweep == 0 ? d_first_buf : d_later_buf)[i] = d;
                }
    }
    // level schedule per class
    long long nnz_total = rp[n];
    // exact GS depth launches hold few rows each: a wave per row pays from short lengths on
    sp.long_rows = n > 0 && nnz_total >= (long long)std::min(32, wave_row_min()) * n;
    std::atomic<bool> coupled{false};   // any same-class off-diagonal entry at all?
    parallel_chunks(n, 1 << 16, [&](int lo, int hi) {
        for (int i = lo; i < hi && !coupled; ++i)
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                const int j = ci[k];
                if (j != i && j < n && cls[j] == cls[i]) {
                    coupled = true;
                    break;
                }
            }
    });
    PhaseTimer pt("plan");
    pt.mark("classes+coupled");
    // red-black levels (no coupling) keep depth 0 everywhere; so do C/F-Jacobi levels, whose
    // passes read only the other iterate (their schedule is never walked by depth)
    if (coupled && kind != SSS_HIP_SMOOTH_JACOBI) {
        for (int i = 0; i < n; ++i) {
            int dep = pushed[i];
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                const int j = ci[k];
                if (j < i && cls[j] == cls[i]) dep = std::max(dep, depth[j] + 1);
            }
            depth[i] = dep;
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                const int j = ci[k];
                if (j > i && j < n && cls[j] == cls[i]) pushed[j] = std::max(pushed[j], dep + 1);
            }
        }
    }
    pt.mark("depth");
    for (int c = 0; c < 2; ++c) {
        PassSchedule &ps = sp.pass[c];
        int maxd = -1;
        for (int i = 0; i < n; ++i)
            if (cls[i] == c) maxd = std::max(maxd, depth[i]);
        ps.depth = maxd + 1;
        ps.h_off.assign(ps.depth + 1, 0);
        for (int i = 0; i < n; ++i)
            if (cls[i] == c) ps.h_off[depth[i] + 1]++;
        for (int l = 0; l < ps.depth; ++l) {
            ps.max_width = std::max(ps.max_width, ps.h_off[l + 1]);
            ps.h_off[l + 1] += ps.h_off[l];
        }
        ps.nrows = ps.depth > 0 ? ps.h_off[ps.depth] : 0;
        std::vector<int> fill(ps.h_off.begin(), ps.h_off.end()), rows(std::max(ps.nrows, 1));
        for (int i = 0; i < n; ++i)
            if (cls[i] == c) rows[fill[depth[i]]++] = i;
        if ((rc = upload_ints(&ps.rows, rows))) return rc;
        ps.compact = kind == SSS_HIP_SMOOTH_JACOBI || ps.depth <= 1;
        if (ps.compact && ps.nrows > 0 && dA && single_diag) {
            // contiguous class?  (relabeled level: F rows first, then C rows)
            int lo = -1, hi = -1;
            bool contiguous = true;
            for (int i = 0; i < n && contiguous; ++i) {
                if (cls[i] != c) continue;
                if (lo < 0) lo = i;
                else if (i != hi) contiguous = false;
                hi = i + 1;
            }
            if (contiguous) {
                // the pass must be a whole number of the level's row blocks
                if (lo == 0 && hi == n) ps.range = true, ps.blo = 0, ps.bhi = dA->nblk;
                else if (lo == 0 && hi == dA->split_row) ps.range = true, ps.blo = 0, ps.bhi = dA->split_blk;
                else if (lo == dA->split_row && hi == n) ps.range = true, ps.blo = dA->split_blk, ps.bhi = dA->nblk;
                ps.lo = lo;
                ps.hi = hi;
            }
            if (ps.range && kind == SSS_HIP_SMOOTH_JACOBI) {
                ps.y = dev_alloc<double>((size_t)(hi - lo));
                if (!ps.y) return hip_fail(hipErrorOutOfMemory, "hipMalloc(y)", __FILE__, __LINE__);
                if (inner > 0) {
                    ps.y2 = dev_alloc<double>((size_t)(hi - lo));
                    if (!ps.y2) return hip_fail(hipErrorOutOfMemory, "hipMalloc(y2)", __FILE__, __LINE__);
                }
            }
        }
        if (ps.compact && ps.nrows > 0 && !ps.range) {
            std::vector<int> crp(1, 0), cci, cmap;
            std::vector<double> cv;
            for (int i = 0; i < n; ++i) {
                if (cls[i] != c) continue;
                cmap.push_back(i);
                for (int k = rp[i]; k < rp[i + 1]; ++k) {
                    cci.push_back(ci[k] == i ? -1 : ci[k]);   // diagonal -> product +0.0 (identity)
                    cv.push_back(v[k]);
                }
                crp.push_back((int)cci.size());
            }
            SSS_MAT sub;
            sub.num_rows = (int)cmap.size();
            sub.num_cols = A.num_cols;
            sub.num_nnzs = (int)cci.size();
            sub.row_ptr = crp.data();
            sub.col_idx = cci.data();
            sub.val = cv.data();
            if ((rc = devcsr_upload(ps.sub, sub))) return rc;
            if ((rc = upload_ints(&ps.map, cmap))) return rc;
            if (kind == SSS_HIP_SMOOTH_JACOBI) {
                ps.y = dev_alloc<double>(cmap.size());
                if (!ps.y) return hip_fail(hipErrorOutOfMemory, "hipMalloc(y)", __FILE__, __LINE__);
            }
        }
    }
    if ((rc = upload_ints(&sp.cls, cls))) return rc;
    t_sched = now();
    // exact GS passes with intra-class chains: one launch per pass where the class is contiguous
    if (kind == SSS_HIP_SMOOTH_EXACT && !gcls && A.num_cols == n) {
        for (int c = 0; c < 2; ++c) {
            PassSchedule &ps = sp.pass[c];
            if (ps.compact || ps.depth <= 1 || ps.nrows == 0) continue;
            int lo = -1, hi = -1;
            bool contiguous = true;
            for (int i = 0; i < n && contiguous; ++i) {
                if (cls[i] != c) continue;
                if (lo < 0) lo = i;
                else if (i != hi) contiguous = false;
                hi = i + 1;
            }
            if (contiguous && (rc = gs_persist_build(ps, A, lo, hi, sp.long_rows))) return rc;
        }
    }
    {   // every pass of a call in one launch (exact GS-CF, both passes on the flow engine; 2 sweeps,
        // SSS_amg_pars_init's pre/post count)
        const char *fe = getenv("SSS_HIP_GS_FUSED");   // 0: per-pass launches (tests compare both)
        if (!(fe && *fe == '0') && kind == SSS_HIP_SMOOTH_EXACT && !gcls && A.num_cols == n && mark &&
            sp.pass[0].gp.engine == 1 && sp.pass[1].gp.engine == 1 &&
            (rc = gs_fused_build(sp.fz, A, dA, sp.pass, cls.data(), 2)))
            return rc;
    }
    t_persist = now();
    if (kind == SSS_HIP_SMOOTH_JACOBI && inner > 0 && sp.pass[0].range == (sp.pass[0].nrows > 0) &&
        sp.pass[1].range == (sp.pass[1].nrows > 0)) {
        sp.inner = inner;
        for (auto &ps : sp.pass) {
            if (ps.nrows == 0) continue;
            const int m = ps.hi - ps.lo;
            const int c = (int)(&ps - sp.pass);
            // L_i: same class, j < i in the global order -- own rows of the pass below i, or
            // (distributed levels) ghost columns of this class owned by lower ranks
            auto lower = [&](int i, int j) { return j < n ? (j >= ps.lo && j < i) : (gcls && gcls[j - n] == c); };
            // two row-parallel passes: count, then fill at the prefix offsets (same order as a
            // sequential build: N_i entries in stored order, then L_i entries in stored order)
            std::vector<int> nrp((size_t)m + 1, 0), lrp((size_t)m + 1, 0), split(m);
            parallel_chunks(m, 1 << 12, [&](int a, int e) {
                for (int q = a; q < e; ++q) {
                    const int i = ps.lo + q;
                    int nn = 0, nl = 0;
                    for (int k = rp[i]; k < rp[i + 1]; ++k) {
                        const int j = ci[k];
                        if (lower(i, j)) ++nl;
                        else if (j != i) ++nn;
                    }
                    nrp[q + 1] = nn + nl;
                    lrp[q + 1] = nl;
                }
            });
            for (int q = 0; q < m; ++q) nrp[q + 1] += nrp[q], lrp[q + 1] += lrp[q];
            pt.mark("ts count");
            HostBuf<int> nci, lci;   // every slot written below (no serial zero-fill)
            HostBuf<double> nv, lv;
            nci.resize((size_t)nrp[m]), lci.resize((size_t)lrp[m]), nv.resize((size_t)nrp[m]), lv.resize((size_t)lrp[m]);
            parallel_chunks(m, 1 << 12, [&](int a, int e) {
                for (int q = a; q < e; ++q) {
                    const int i = ps.lo + q;
                    int o = nrp[q], ol = lrp[q];
                    for (int k = rp[i]; k < rp[i + 1]; ++k) {   // N_i: off-diagonal, not same-class lower
                        const int j = ci[k];
                        if (j != i && !lower(i, j)) nci[o] = j, nv[o] = v[k], ++o;
                    }
                    split[q] = o;
                    for (int k = rp[i]; k < rp[i + 1]; ++k) {   // L_i
                        const int j = ci[k];
                        if (lower(i, j)) {
                            nci[o] = j, nv[o] = v[k], ++o;
                            lci[ol] = j, lv[ol] = v[k], ++ol;
                        }
                    }
                }
            });
            auto mk = [&](std::vector<int> &r, HostBuf<int> &c, HostBuf<double> &w) {
                SSS_MAT M;
                M.num_rows = m;
                M.num_cols = A.num_cols;
                M.num_nnzs = (int)c.size();
                M.row_ptr = r.data();
                M.col_idx = c.data();
                M.val = w.data();
                return M;
            };
            pt.mark("ts fill");
            SSS_MAT Mn = mk(nrp, nci, nv), Ml = mk(lrp, lci, lv);
            std::vector<int> seg(split);   // absolute [N_i | L_i] cut of each row of Mn
            // read by the ts_* kernels only: merged groups, or the column ELL
            const int tenc = (enc & ~kEncDict) | kEncMergedOnly;
            if ((rc = devcsr_upload(ps.ts_nl, Mn, -1, tenc, seg.data())) || (rc = devcsr_upload(ps.ts_lo, Ml, -1, tenc)))
                return rc;
            pt.mark("ts upload");
            if ((rc = upload_ints(&ps.ts_split, split))) return rc;
            ps.ts_P = dev_alloc<double>((size_t)m);
            if (!ps.ts_P) return hip_fail(hipErrorOutOfMemory, "hipMalloc(P)", __FILE__, __LINE__);
        }
    }
    t_two = now();
    if (sp.pass[0].range || sp.pass[1].range)
        if ((rc = upload_ints(&sp.diag_pos, diag_pos))) return rc;
    const char *nc = getenv("SSS_HIP_NOCOPY");   // 0: C/F-Jacobi through per-pass copies (tests)
    if (!(nc && *nc == '0') && kind == SSS_HIP_SMOOTH_JACOBI && !gcls && A.num_cols == n) {
        const PassSchedule &F = sp.pass[0], &Cp = sp.pass[1];
        const bool f_ok = F.nrows == 0 || (F.range && F.lo == 0), c_ok = Cp.nrows == 0 || (Cp.range && Cp.hi == n);
        const int cs = F.nrows > 0 ? F.hi : 0;
        if (f_ok && c_ok && (Cp.nrows == 0 || Cp.lo == cs) && (F.nrows > 0 || Cp.nrows > 0)) {
            sp.csplit = cs;
            sp.x2 = dev_alloc<double>((size_t)n);
            if (!sp.x2) return hip_fail(hipErrorOutOfMemory, "hipMalloc(x2)", __FILE__, __LINE__);
        }
    }
    sp.own_diag = all_diag && single_diag && !(tz && *tz == '0');
    {
        const char *zz = getenv("SSS_HIP_ZERO_FIRST");   // 0: run the first pass on a zero x in full (tests)
        std::atomic<bool> fin{!(zz && *zz == '0')};
        if (fin)
            parallel_chunks(n, 1 << 16, [&](int lo, int hi) {
                for (int k = rp[lo]; k < rp[hi] && fin; ++k)
                    if (!std::isfinite(v[k])) fin = false;
            });
        sp.finite = fin;
    }
    {
        const char *dz = getenv("SSS_HIP_DEAD_PROLONG");   // 0: always prolong into every row (tests)
        const PassSchedule &F = sp.pass[0];
        bool ok = !(dz && *dz == '0') && kind != SSS_HIP_SMOOTH_JACOBI && F.range && F.lo == 0 && F.nrows > 0 &&
                  F.depth <= 1 && single_diag;
        for (int i = F.lo; ok && i < F.hi; ++i)
            ok = std::fabs(d_first[i]) > SMALLFLOAT && std::fabs(all_diag ? d_first[i] : d_later[i]) > SMALLFLOAT;
        sp.f_overwritten = ok;
    }
    const char *fz = getenv("SSS_HIP_FUSE_RESID");
    const char *pz = getenv("SSS_HIP_PEND_F");   // 0: never precompute the first F pass (tests)   // 0: never fuse (tests compare both paths)
    if (!(fz && *fz == '0') && kind != SSS_HIP_SMOOTH_JACOBI && dA && !dA->wave_rows && !dA->vec_rows && all_diag && single_diag &&
        dA->split_row > 0 &&
        dA->split_row < n && sp.pass[0].range && sp.pass[1].range && sp.pass[0].lo == 0 &&
        sp.pass[0].hi == dA->split_row && sp.pass[1].lo == dA->split_row && sp.pass[1].hi == n) {
        // the MODE 2 / 3 passes have no long-row path: every block of the pass within one tile (the
        // ELL formats take one row per thread and rows of at most 32 entries)
        std::vector<int> blk;
        const bool ell = dA->dv_ell || dA->dv_xell;
        if (!ell) build_row_blocks(rp, n, blk, dA->split_row);
        bool short_blocks = true;
        for (int q = dA->split_blk; !ell && q < dA->nblk && short_blocks; ++q)
            short_blocks = rp[blk[q + 1]] - rp[blk[q]] <= kTileEntries;
        sp.fuse_resid = short_blocks;
        bool f_short = true;
        for (int q = 0; !ell && q < dA->split_blk && f_short; ++q) f_short = rp[blk[q + 1]] - rp[blk[q]] <= kTileEntries;
        sp.pend_ok = short_blocks && f_short && sp.f_overwritten && !(pz && *pz == '0');
    }
    if (timing)
        fprintf(stderr, "[sss_hip]   smoother plan n=%d: schedule %.2f s, one-launch GS %.2f s, two-stage %.2f s, rest %.2f s\n",
                n, t_sched - t0, t_persist - t_sched, t_two - t_persist, now() - t_two);
    if (kind == SSS_HIP_SMOOTH_JACOBI || all_diag) {   // Jacobi: row's own diagonal
        if ((rc = upload_doubles(&sp.d_first, last_diag))) return rc;
        sp.d_later = sp.d_first;
    } else {
        if ((rc = upload_doubles(&sp.d_first, d_first_buf))) return rc;
        if ((rc = upload_doubles(&sp.d_later, d_later_buf))) return rc;
    }
    return 0;
}

void smoother_free(SmootherPlan &sp)
{
    for (auto &ps : sp.pass) {
        dev_free(ps.rows);
        devcsr_free(ps.sub);
        dev_free(ps.map);
        dev_free(ps.y);
        dev_free(ps.y2);
        devcsr_free(ps.ts_nl);
        devcsr_free(ps.ts_lo);
        dev_free(ps.ts_split);
        dev_free(ps.ts_P);
        gs_persist_free(ps);
    }
    gs_fused_free(sp.fz);
    if (sp.d_later != sp.d_first) dev_free(sp.d_later);
    dev_free(sp.d_first);
    dev_free(sp.nd_first);
    dev_free(sp.nd_later);
    dev_free(sp.cls);
    dev_free(sp.diag_pos);
    dev_free(sp.x2);
    sp = SmootherPlan();
}

// ---- kernels -------------------------------------------------------------------------------
// exact GS, one thread per row of the current depth.  NAT: natural-order GS (Solve/SSS_smooth.c:
// 90-137), x_i = t * d with d the carried reciprocal of the diagonal, written unconditionally.
template <bool NAT>
__global__ __launch_bounds__(kBlock) void gs_depth_thread(const int *__restrict__ rows, int cnt,
                                                          const int *__restrict__ rp, const int *__restrict__ ci,
                                                          const double *__restrict__ v, const double *__restrict__ b,
                                                          double *x, const double *__restrict__ deff)
{
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= cnt) return;
    const int i = rows[t];
    double acc = b[i];
    for (int k = rp[i]; k < rp[i + 1]; ++k) {
        const int j = ci[k];
        if (j != i) acc -= v[k] * x[j];
    }
    const double d = deff[i];
    if (NAT) x[i] = acc * d;
    else if (fabs(d) > SMALLFLOAT) x[i] = acc / d;
}

// exact GS on long rows: four rows of the current depth per workgroup, one per wave; lanes
// gather the products, lane 0 subtracts them in CSR order (sss_spmv_dev.hpp wave_row_chain).
template <bool NAT>
__global__ __launch_bounds__(kBlock) void gs_depth_wave(const int *__restrict__ rows, int cnt,
                                                        const int *__restrict__ rp, const int *__restrict__ ci,
                                                        const double *__restrict__ v, const double *__restrict__ b,
                                                        double *x, const double *__restrict__ deff)
{
    __shared__ __attribute__((aligned(16))) double strips[4][kWaveStage];
    const int wave = threadIdx.x >> 6;
    const int t = blockIdx.x * 4 + wave;
    if (t >= cnt) return;
    const int i = rows[t];
    const double acc = wave_row_chain<true>(
        rp[i], rp[i + 1], ci, v, [&](int c, double a) { return c == i ? 0.0 : a * x[c]; }, b[i], strips[wave]);
    if ((threadIdx.x & 63) == 0) {
        const double d = deff[i];
        if (NAT) x[i] = acc * d;
        else if (fabs(d) > SMALLFLOAT) x[i] = acc / d;
    }
}

// Independent-row pass over the class-compacted CSR: GS with depth 1 (in place) or the
// relaxation half of a C/F-Jacobi pass (into y, scattered afterwards).
template <bool INPLACE>
__global__ __launch_bounds__(kBlock) void relax_compact(const int *__restrict__ blk, const int *__restrict__ rp,
                                                        const int *__restrict__ ci, const double *__restrict__ v,
                                                        const int *__restrict__ map, const double *__restrict__ b,
                                                        double *x, double *__restrict__ y,
                                                        const double *__restrict__ deff)
{
    __shared__ SpmvSmem sm;
    csr_block_relax(blk, rp, ci, v, map, b, x, sm, [&](int r, int i, double acc) {
        const double d = deff[i];
        if (INPLACE) {
            if (fabs(d) > SMALLFLOAT) x[i] = acc / d;
        } else {
            y[r] = fabs(d) > SMALLFLOAT ? acc / d : x[i];
        }
    });
}

template <bool INPLACE>
__global__ __launch_bounds__(kBlock) void relax_wave(int m, const int *__restrict__ rp, const int *__restrict__ ci,
                                                     const double *__restrict__ v, const int *__restrict__ map,
                                                     const double *__restrict__ b, double *x, double *__restrict__ y,
                                                     const double *__restrict__ deff)
{
    __shared__ __attribute__((aligned(16))) double strips[4][kWaveStage];
    const int wave = threadIdx.x >> 6;
    const int r = xcd_bid() * 4 + wave;
    if (r >= m) return;
    const int i = map[r];
    const double acc = wave_row_chain<true>(
        rp[r], rp[r + 1], ci, v, [&](int c, double a) { return (c < 0 || c == i) ? 0.0 : a * x[c]; }, b[i],
        strips[wave]);
    if ((threadIdx.x & 63) == 0) {
        const double d = deff[i];
        if (INPLACE) {
            if (fabs(d) > SMALLFLOAT) x[i] = acc / d;
        } else {
            y[r] = fabs(d) > SMALLFLOAT ? acc / d : x[i];
        }
    }
}

// Class pass over rows [lo, hi) of a relabeled level, blocks [blo, ...) of its own CSR.
//   MODE 0: GS-CF pass of depth 1, in place (x[r] = t / d).
//   MODE 1: C/F-Jacobi pass / two-stage stage 0: y[r - lo] = t / d, every x from before the pass.
//   MODE 3: the residual of the row with x unchanged (rr, partial, as the residual SpMV) and the
//           GS value the pass's MODE 0 would write, into y[r - lo] (SmootherPlan::pend_ok).
//   MODE 2: MODE 0, then the residual of the updated row (ResidFuse, sss_engine.hpp):
//           rr[r] = b_r - (sum of a_k x_k in stored order from 0.0), the diagonal product formed
//           with the new x_r -- exactly the residual SpMV's chain, since in a depth-1 pass no
//           other product of the row changes; per-block sums of squares into partial[bid].
// t = b_r - sum over off-diagonal entries in stored order (diag_pos skips the diagonal); rows with
// |d| <= 1e-20 keep their value.
// Dictionary ELL rows (DICT == 2): the same per-row arithmetic, the row's products in registers in
// stored (slot) order instead of staged in LDS.
template <int MODE, int W>
__device__ __forceinline__ void relax_range_ell(int blo, const int2 *__restrict__ blk, int lo,
                                                const double *__restrict__ b, double *x, double *__restrict__ y,
                                                const double *__restrict__ deff, double *__restrict__ rr,
                                                double *__restrict__ partial, XSrc xs, const DevDict &dt)
{
    constexpr int RPT = kEllRpt;
    __shared__ EllSmem es[RPT];
    const int g = (int)blockIdx.x;
    unsigned w[RPT][W / 4];
    double br[RPT], dr[RPT];
    int r[RPT];
    bool live[RPT], valid[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {   // every row's codes, b and divisor in flight across the barrier
        const int bid = blo + g * RPT + j;
        valid[j] = bid < dt.bend;
        live[j] = false;
        br[j] = dr[j] = 0.0;
        r[j] = 0;
#pragma unroll
        for (int t = 0; t < W / 4; ++t) w[j][t] = 0u;
        if (valid[j]) {
            const int2 ba = blk[bid], be = blk[bid + 1];
            r[j] = ba.x + (int)threadIdx.x;
            live[j] = r[j] < be.x;
            if (live[j]) {
                ell_codes<W>(dt.ell, r[j], w[j]);
                br[j] = b[r[j]];
                if (deff) dr[j] = deff[r[j]];
            }
            ell_load_dicts_nosync(dt, bid, es[j]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        double sq = 0.0;
        if (live[j]) {
            const int rj = r[j];
            double p[W];
            int dsl;
            double dv;
            // the pass's own x_r only in MODE 3 (the residual of the row with x unchanged)
            const int len = ell_decode<W, MODE == 3>(w[j], rj, es[j], [&](int c) -> double { return xs(c); }, p, dsl, dv);
            const double acc = dsl < 0 ? ell_sub(br[j], p, 0, len) : ell_sub(ell_sub(br[j], p, 0, dsl), p, dsl + 1, len);
            const double d = deff ? dr[j] : dv;
            if constexpr (MODE == 2) {
                const double xn = fabs(d) > SMALLFLOAT ? acc / d : x[rj];
                if (fabs(d) > SMALLFLOAT) x[rj] = xn;
                double t = ell_add(0.0, p, 0, dsl);
                t += d * xn;
                t = ell_add(t, p, dsl + 1, len);
                const double out = br[j] + t * -1.0;
                rr[rj] = out;
                sq = out * out;
            } else if constexpr (MODE == 3) {
                const double out = br[j] + ell_add(0.0, p, 0, len) * -1.0;
                rr[rj] = out;
                sq = out * out;
                y[rj - lo] = fabs(d) > SMALLFLOAT ? acc / d : x[rj];
            } else if constexpr (MODE == 1) {
                y[rj - lo] = fabs(d) > SMALLFLOAT ? acc / d : xs(rj);
            } else {
                if (fabs(d) > SMALLFLOAT) x[rj] = acc / d;
            }
        }
        if constexpr (MODE >= 2) {
            if (partial && valid[j]) {   // (valid is uniform over the workgroup)
                const double t = block_sum(sq, es[j].red);
                if (threadIdx.x == 0) partial[blo + g * RPT + j] = t;
            }
        }
    }
}

// relax_range_ell for W = 8 with two consecutive rows per thread (sss_spmv_dev.hpp ell_pair_rows):
// every row's arithmetic exactly as relax_range_ell's, x / y / rr / b moved as 16-byte pairs.
template <int MODE>
__device__ __forceinline__ void relax_range_ell2(int blo, const int2 *__restrict__ blk, int lo,
                                                 const double *__restrict__ b, double *x, double *__restrict__ y,
                                                 const double *__restrict__ deff, double *__restrict__ rr,
                                                 double *__restrict__ partial, XSrc xs, const DevDict &dt)
{
    __shared__ EllSmem es[2];
    const int g = (int)blockIdx.x;
    const EllPairRows pr = ell_pair_rows(blk, blo + 2 * g, dt.bend);
    unsigned w[2][2];
    double br[2], dr[2] = {0.0, 0.0};
    ell_pair_codes(dt.ell, pr, w);   // every row's codes, b and divisor in flight across the barrier
    pair_load(b, pr.r, pr.l0, pr.l1, br);
    if (deff) pair_load(deff, pr.r, pr.l0, pr.l1, dr);
    if (pr.v0) ell_load_dicts_nosync(dt, pr.b0, es[0]);
    if (pr.v1) ell_load_dicts_nosync(dt, pr.b0 + 1, es[1]);
    __syncthreads();
    double xo[2] = {0.0, 0.0}, ro[2] = {0.0, 0.0}, sq[2] = {0.0, 0.0};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int rj = pr.r + i;
        if (!(i == 0 ? pr.l0 : pr.l1)) continue;
        const int j = rj < pr.mid ? 0 : 1;
        double p[8];
        int dsl;
        double dv;
        const int len = ell_decode<8, MODE == 3>(w[i], rj, es[j], [&](int c) -> double { return xs(c); }, p, dsl, dv);
        const double acc = dsl < 0 ? ell_sub(br[i], p, 0, len) : ell_sub(ell_sub(br[i], p, 0, dsl), p, dsl + 1, len);
        const double d = deff ? dr[i] : dv;
        if constexpr (MODE == 2) {
            const double xn = fabs(d) > SMALLFLOAT ? acc / d : x[rj];
            xo[i] = xn;
            double t = ell_add(0.0, p, 0, dsl);
            t += d * xn;
            t = ell_add(t, p, dsl + 1, len);
            ro[i] = br[i] + t * -1.0;
            sq[j] += ro[i] * ro[i];
        } else if constexpr (MODE == 3) {
            ro[i] = br[i] + ell_add(0.0, p, 0, len) * -1.0;
            sq[j] += ro[i] * ro[i];
            xo[i] = fabs(d) > SMALLFLOAT ? acc / d : x[rj];
        } else if constexpr (MODE == 1) {
            xo[i] = fabs(d) > SMALLFLOAT ? acc / d : xs(rj);
        } else {
            xo[i] = fabs(d) > SMALLFLOAT ? acc / d : x[rj];   // (a row with |d| <= 1e-20 keeps its value)
        }
    }
    if constexpr (MODE == 0 || MODE == 2) pair_store(x, pr.r, pr.l0, pr.l1, xo);
    if constexpr (MODE == 1 || MODE == 3) pair_store(y, pr.r - lo, pr.l0, pr.l1, xo);
    if constexpr (MODE >= 2) pair_store(rr, pr.r, pr.l0, pr.l1, ro);
    if constexpr (MODE >= 2) {
        // per-block sums of squares in the residual SpMV's order (one row per thread, block_sum's
        // fixed tree): each row's square goes through LDS to the thread that row has there, so the
        // norm is bitwise the unfused residual's (tests/test_gpu_parity.py test_fused_residual_bitwise)
        __shared__ double sqrow[2 * kBlock];
        if (partial && pr.v0) {   // (uniform over the workgroup)
            const int ra = pr.r - 2 * (int)threadIdx.x;
            if (pr.l0) sqrow[pr.r - ra] = ro[0] * ro[0];
            if (pr.l1) sqrow[pr.r + 1 - ra] = ro[1] * ro[1];
            __syncthreads();
            const int n0 = pr.mid - ra, n1 = pr.v1 ? ell_block_rows(pr) - n0 : 0;
            const double t0 = block_sum((int)threadIdx.x < n0 ? sqrow[threadIdx.x] : 0.0, es[0].red);
            if (threadIdx.x == 0) partial[pr.b0] = t0;
            if (pr.v1) {
                const double t1 = block_sum((int)threadIdx.x < n1 ? sqrow[n0 + threadIdx.x] : 0.0, es[1].red);
                if (threadIdx.x == 0) partial[pr.b0 + 1] = t1;
            }
        }
        (void)sq;
    }
}

// Column ELL rows (DICT = kXell + W): relax_range_ell's per-row arithmetic, one row block per
// workgroup, the row's products in registers from its explicit-column codes.
template <int MODE, int W>
__device__ __forceinline__ void relax_range_xell(int blo, const int2 *__restrict__ blk, int lo,
                                                 const double *__restrict__ b, double *x, double *__restrict__ y,
                                                 const double *__restrict__ deff, double *__restrict__ rr,
                                                 double *__restrict__ partial, XSrc xs, const DevDict &dt)
{
    __shared__ XellSmem es;
    const int bid = blo + (int)blockIdx.x;
    const bool valid = bid < dt.bend;
    unsigned w[W];
    double br = 0.0, dr = 0.0;
    int r = 0;
    bool live = false;
#pragma unroll
    for (int t = 0; t < W; ++t) w[t] = 0xffffffffu;
    if (valid) {   // the row's codes, b and divisor in flight across the barrier
        const int2 ba = blk[bid], be = blk[bid + 1];
        r = ba.x + (int)threadIdx.x;
        live = r < be.x;
        if (live) {
            xell_codes<W>(dt.xell, r, w);
            br = b[r];
            if (deff) dr = deff[r];
        }
        xell_load_dict_nosync(dt, bid, es);
    }
    __syncthreads();
    double sq = 0.0;
    if (live) {
        double xv[W];
        int dsl;
        unsigned dcode;
        const int len = xell_gather<W, MODE == 3>(w, r, dt.xshift, [&](int c) -> double { return xs(c); }, xv, dsl, dcode);
        const double acc = dsl < 0 ? xell_sub(br, w, xv, es, dt.xshift, 0, len)
                                   : xell_sub(xell_sub(br, w, xv, es, dt.xshift, 0, dsl), w, xv, es, dt.xshift, dsl + 1, len);
        const double dv = dsl < 0 ? 0.0 : es.vd[dcode >> dt.xshift];
        const double d = deff ? dr : dv;
        if constexpr (MODE == 2) {
            const double xn = fabs(d) > SMALLFLOAT ? acc / d : x[r];
            if (fabs(d) > SMALLFLOAT) x[r] = xn;
            double t = xell_add(0.0, w, xv, es, dt.xshift, 0, dsl);
            t += d * xn;
            t = xell_add(t, w, xv, es, dt.xshift, dsl + 1, len);
            const double out = br + t * -1.0;
            rr[r] = out;
            sq = out * out;
        } else if constexpr (MODE == 3) {
            const double out = br + xell_add(0.0, w, xv, es, dt.xshift, 0, len) * -1.0;
            rr[r] = out;
            sq = out * out;
            y[r - lo] = fabs(d) > SMALLFLOAT ? acc / d : x[r];
        } else if constexpr (MODE == 1) {
            y[r - lo] = fabs(d) > SMALLFLOAT ? acc / d : xs(r);
        } else {
            if (fabs(d) > SMALLFLOAT) x[r] = acc / d;
        }
    }
    if constexpr (MODE >= 2) {
        if (partial && valid) {   // (valid is uniform over the workgroup)
            const double t = block_sum(sq, es.red);
            if (threadIdx.x == 0) partial[bid] = t;
        }
    }
}

template <int MODE, int DICT = 0>   // DICT: with_tile_kind (8/16/32: dictionary ELL, kXell + W: column ELL)
__device__ __forceinline__ void relax_range_body(int blo, const int2 *__restrict__ blk, const int *__restrict__ rp,
                                                      const int *__restrict__ ci, const double *__restrict__ v,
                                                      const int *__restrict__ diag_pos, int lo,
                                                      const double *__restrict__ b, double *x,
                                                      const double *__restrict__ yp, double *__restrict__ y,
                                                      const double *__restrict__ deff, const unsigned *__restrict__ pk,
                                                      const double *__restrict__ pv, const int2 *__restrict__ pb,
                                                      double *__restrict__ rr, double *__restrict__ partial, XSrc xs,
                                                      DevDict dt = DevDict())
{
    if constexpr (DICT >= kXell) {
        relax_range_xell<MODE, DICT - kXell>(blo, blk, lo, b, x, y, deff, rr, partial, xs, dt);
    } else if constexpr (DICT == 8 && kEllPairs) {
        relax_range_ell2<MODE>(blo, blk, lo, b, x, y, deff, rr, partial, xs, dt);
    } else if constexpr (DICT >= 8) {
        relax_range_ell<MODE, DICT>(blo, blk, lo, b, x, y, deff, rr, partial, xs, dt);
    } else {
    __shared__ SpmvSmem sm;
    __shared__ std::conditional_t<DICT != 0, DictSmem, char> dsm;
    DictSmem *ds = nullptr;
    if constexpr (DICT != 0) ds = &dsm;
    const int bid = blo + xcd_bid();
    const int2 ba = blk[bid], be = blk[bid + 1];
    const int r0 = ba.x, r1 = be.x, k0 = ba.y, k1 = be.y;
    auto fetch = [&](int c) -> double { return xs(c); };
    // deff null: the plan's divisor is each row's own diagonal, staged from the sorted tile
    auto dval = [&](int r) -> double { return deff ? deff[r] : sm.d[r - r0]; };
    auto finish = [&](int r, double acc) {
        const double d = dval(r);
        if (MODE != 1) {
            if (fabs(d) > SMALLFLOAT) x[r] = acc / d;
        } else {
            y[r - lo] = fabs(d) > SMALLFLOAT ? acc / d : xs(r);
        }
    };
    if (k1 - k0 <= kTileEntries) {
        const int r = r0 + (int)threadIdx.x;
        int a = 0, e = 0, dp = -1;
        double acc = 0.0, br = 0.0;
        if (r < r1) a = rp[r] - k0, e = rp[r + 1] - k0, dp = diag_pos[r], br = b[r];   // ahead of the tile
        stage_any(sm.v, k0, k1, ci, v, pk, pv, pb, bid, r0, deff ? (double *)nullptr : sm.d, fetch, dt, ds, r1, rp);
        __syncthreads();
        double sq = 0.0;
        if (r < r1) {
            acc = br;
            if (dp < 0) acc = chain_sub(acc, sm.v, a, e);
            else {
                acc = chain_sub(acc, sm.v, a, dp - k0);
                acc = chain_sub(acc, sm.v, dp - k0 + 1, e);
            }
            if constexpr (MODE == 2) {   // plan guarantees one diagonal per row, deff = a_rr
                const double d = dval(r);
                const double xn = fabs(d) > SMALLFLOAT ? acc / d : x[r];
                if (fabs(d) > SMALLFLOAT) x[r] = xn;
                double s = chain_add(0.0, sm.v, a, dp - k0);
                s += d * xn;
                s = chain_add(s, sm.v, dp - k0 + 1, e);
                const double out = br + s * -1.0;
                rr[r] = out;
                sq = out * out;
            } else if constexpr (MODE == 3) {   // residual of the row (x unchanged) + its GS value
                const double out = br + chain_add(0.0, sm.v, a, e) * -1.0;
                rr[r] = out;
                sq = out * out;
                const double d = dval(r);
                y[r - lo] = fabs(d) > SMALLFLOAT ? acc / d : x[r];
            } else {
                finish(r, acc);
            }
        }
        if constexpr (MODE >= 2) {
            if (partial) {
                const double t = block_sum(sq, sm.red);
                if (threadIdx.x == 0) partial[bid] = t;
            }
        }
    } else if constexpr (MODE < 2) {   // MODE 2 / 3 plans have no long-row block
        const int r = r0, dp = diag_pos[r];
        double acc = b[r];
        for (int base = k0; base < k1; base += kTileEntries) {
            const int m = min(kTileEntries, k1 - base);
            stage_any(sm.v, base, base + m, ci, v, pk, pv, pb, bid, r0, deff ? (double *)nullptr : sm.d, fetch, dt, ds,
                      r1, rp);
            __syncthreads();
            if (dt.tree_long) {   // free order: acc -= tree sum of the chunk's off-diagonal products
                if (threadIdx.x == 0 && dp >= base && dp < base + m) sm.v[dp - base] = 0.0;
                __syncthreads();
                const double c = block_tree_sum(sm.v, 0, m, sm.red);
                if (threadIdx.x == 0) acc -= c;
            } else if (threadIdx.x == 0) {
                if (dp >= base && dp < base + m) {
                    acc = chain_sub(acc, sm.v, 0, dp - base);
                    acc = chain_sub(acc, sm.v, dp - base + 1, m);
                } else {
                    acc = chain_sub(acc, sm.v, 0, m);
                }
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) finish(r, acc);
    }
    }
}

#define SSS_RELAX_ARGS                                                                                          \
    int blo, const int2 *__restrict__ blk, const int *__restrict__ rp, const int *__restrict__ ci,                 \
        const double *__restrict__ v, const int *__restrict__ diag_pos, int lo, const double *__restrict__ b,      \
        double *x, const double *__restrict__ yp, double *__restrict__ y, const double *__restrict__ deff,          \
        const unsigned *__restrict__ pk, const double *__restrict__ pv, const int2 *__restrict__ pb,               \
        double *__restrict__ rr, double *__restrict__ partial, XSrc xs, DevDict dt
#define SSS_RELAX_PASS blo, blk, rp, ci, v, diag_pos, lo, b, x, yp, y, deff, pk, pv, pb, rr, partial, xs, dt
template <int MODE, int DICT = 0>
__global__ __launch_bounds__(kBlock) void relax_range(SSS_RELAX_ARGS)
{
    relax_range_body<MODE, DICT>(SSS_RELAX_PASS);
}
// The tile paths (plain / sorted / dictionary tiles, K < 8) held to 5 waves per SIMD: the value-
// dictionary tiles of level 1 otherwise take 107 VGPRs (4 waves per SIMD, 14 resident per CU in
// profiles/r03_kernels_sq_pmc_400.txt) and wait on memory 70 % of their cycles.  Measured at
// 400^3 (tools/gpu/ab.sh): level-1 smoothing 4.61 -> 4.23 ms per V-cycle at 5 waves (96 VGPRs);
// 6 waves (the LDS limit) spill to scratch and take 6.90 ms.
template <int MODE, int DICT = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5, 8))) void relax_range_occ(SSS_RELAX_ARGS)
{
    relax_range_body<MODE, DICT>(SSS_RELAX_PASS);
}
// relax_range / relax_range_occ over the row blocks [blo, blo + nb): one workgroup per block, or
// per kEllRpt blocks on dictionary ELL (K >= 8)
template <int M, int K, class... Args>
static void launch_relax_range(int blo, int nb, hipStream_t s, DevDict dt, Args... args)
{
    if constexpr (K < 8) {
        hipLaunchKernelGGL((relax_range_occ<M, K>), dim3(nb), dim3(kBlock), 0, s, blo, args..., dt);
    } else {
        dt.bend = blo + nb;
        hipLaunchKernelGGL((relax_range<M, K>), dim3((nb + rows_per_wg(K) - 1) / rows_per_wg(K)), dim3(kBlock), 0, s, blo,
                           args..., dt);
    }
}

// relax_range for long-row levels: one wave per row (rows lo + 4 * blockIdx.x + wave).  The
// diagonal (single per row on range levels) contributes an exact 0.0 to the chain.
// TREE: free sum order (DevCSR::vec_rows), t = b_r - (tree sum of the off-diagonal products).
template <int MODE, bool TREE>
__global__ __launch_bounds__(kBlock) void relax_range_wave(int lo, int hi, const int *__restrict__ rp,
                                                           const int *__restrict__ ci, const double *__restrict__ v,
                                                           const double *__restrict__ b, double *x,
                                                           const double *__restrict__ yp, double *__restrict__ y,
                                                           const double *__restrict__ deff, XSrc xs)
{
    __shared__ __attribute__((aligned(16))) double strips[TREE ? 1 : 4][TREE ? 1 : kWaveStage];
    const int wave = threadIdx.x >> 6;
    const int r = lo + xcd_bid() * 4 + wave;
    if (r >= hi) return;
    auto prod = [&](int c, double a) -> double { return c == r ? 0.0 : a * (MODE == 1 ? xs(c) : x[c]); };
    const double acc = TREE ? b[r] - wave_row_sum(rp[r], rp[r + 1], ci, v, prod)
                            : wave_row_chain<true>(rp[r], rp[r + 1], ci, v, prod, b[r], strips[TREE ? 0 : wave]);
    if ((threadIdx.x & 63) == 0) {
        const double d = deff[r];
        if (MODE == 0) {
            if (fabs(d) > SMALLFLOAT) x[r] = acc / d;
        } else {
            y[r - lo] = fabs(d) > SMALLFLOAT ? acc / d : xs(r);
        }
    }
}

// ---- two-stage GS-CF (oracle: ora_cf_twostage) ----------------------------------------------
// Stage 0 over the reordered pass rows [N_i | L_i] (local row q = global lo + q):
//   P_q = b - sum_{N_i} a x;  y_q = (P_q - sum_{L_i} a x) / d   (x from before the pass)
template <int PATH>   // 0 tile, 1 wave chain, 2 wave tree (free order)
__global__ __launch_bounds__(kBlock) void ts_stage0(int lo, DevCSR M, const int *__restrict__ split,
                                                    const double *__restrict__ b, XSrc x,
                                                    const double *__restrict__ deff, double *__restrict__ P,
                                                    double *__restrict__ y)
{
    auto finish = [&](int q, double acc) {
        const int r = lo + q;
        const double d = deff[r];
        y[q] = fabs(d) > SMALLFLOAT ? acc / d : x(r);
    };
    if constexpr (PATH >= kXell) {   // column ELL rows of width PATH - kXell: one thread per row
        constexpr int W = PATH - kXell;
        __shared__ XellSmem es;
        const int bq = blockIdx.x;
        const int2 ba = M.bk[bq], be = M.bk[bq + 1];
        const int q = ba.x + (int)threadIdx.x;
        const bool live = q < be.x;
        unsigned w[W];
        double bq_v = 0.0, dq = 0.0;
        int sp = 0;
#pragma unroll
        for (int t = 0; t < W; ++t) w[t] = 0xffffffffu;
        if (live) {   // the row's codes, b, divisor and its [N | L] cut in flight across the barrier
            xell_codes<W>(M.dv_xell, q, w);
            bq_v = b[lo + q];
            dq = deff[lo + q];
            sp = split[q] - M.rp[q];
        }
        {
            const int4 pq4 = M.dv_pd[bq];
            for (int t = threadIdx.x; t < pq4.w; t += kBlock) es.vd[t] = M.dv_vd[pq4.z + t];
        }
        __syncthreads();
        if (live) {
            double xv[W];
            int ds;
            const int len = xell_gather<W>(w, -1, M.xell_shift, [&](int c) -> double { return x(c); }, xv, ds);
            const double Pq = xell_sum_bf<true>(bq_v, w, xv, es, M.xell_shift, 0, sp);
            P[q] = Pq;
            const double acc = xell_sum_bf<true>(Pq, w, xv, es, M.xell_shift, sp, len);
            y[q] = fabs(dq) > SMALLFLOAT ? acc / dq : x(lo + q);   // finish() with the divisor loaded early
        }
        return;
    } else if constexpr (PATH >= 3) {   // merged row groups, G = PATH, M.mg_W waves per group
        constexpr int G = PATH;
        __shared__ double red[8 * G];
        int g = 0, u = 0;
        double n_sum = 0.0, l_sum = 0.0;
        if (merged_block<G, 2>(M.mg_gp, M.mg_ng, M.mg_W, M.mg_k, M.mg_v, [&](int c) -> double { return x(c); }, red, g, u,
                               n_sum, l_sum)) {
            const int q = g * G + u;
            if (q < M.n) {
                const double Pq = b[lo + q] - n_sum;
                P[q] = Pq;
                finish(q, Pq - l_sum);
            }
        }
        return;
    } else if constexpr (PATH == 2) {
        const int q = xcd_bid() * 4 + (threadIdx.x >> 6);
        if (q >= M.n) return;
        auto prod = [&](int c, double a) { return a * x(c); };
        const int a = M.rp[q], sp = split[q], e = M.rp[q + 1];
        const double Pq = b[lo + q] - wave_row_sum(a, sp, M.ci, M.v, prod);
        const double acc = Pq - wave_row_sum(sp, e, M.ci, M.v, prod);
        if ((threadIdx.x & 63) == 0) {
            P[q] = Pq;
            finish(q, acc);
        }
        return;
    } else if constexpr (PATH == 1) {
        __shared__ __attribute__((aligned(16))) double strips[4][kWaveStage];
        const int wave = threadIdx.x >> 6, q = xcd_bid() * 4 + wave;
        if (q >= M.n) return;
        auto prod = [&](int c, double a) { return a * x(c); };
        const int a = M.rp[q], sp = split[q], e = M.rp[q + 1];
        double acc = wave_row_chain<true>(a, sp, M.ci, M.v, prod, b[lo + q], strips[wave]);
        acc = __shfl(acc, 0, 64);
        if ((threadIdx.x & 63) == 0) P[q] = acc;
        acc = wave_row_chain<true>(sp, e, M.ci, M.v, prod, acc, strips[wave]);
        if ((threadIdx.x & 63) == 0) finish(q, acc);
        return;
    } else {
        __shared__ SpmvSmem sm;
        const int bq = xcd_bid();
        const BlockBounds bb = block_bounds(M.bk, M.rp, bq);
        const int q0 = bb.r0, q1 = bb.r1, k0 = bb.k0, k1 = bb.k1;
        if (k1 - k0 <= kTileEntries) {
            const int q = q0 + (int)threadIdx.x;
            int a = 0, sp = 0, e = 0;
            double acc = 0.0;
            if (q < q1) a = M.rp[q] - k0, sp = split[q] - k0, e = M.rp[q + 1] - k0, acc = b[lo + q];
            stage_any(sm.v, k0, k1, M.ci, M.v, M.pk, M.pv, M.pb, bq, q0, (double *)nullptr, [&](int c) -> double { return x(c); });
            __syncthreads();
            if (q < q1) {
                acc = chain_sub(acc, sm.v, a, sp);
                P[q] = acc;
                acc = chain_sub(acc, sm.v, sp, e);
                finish(q, acc);
            }
        } else {   // one long row, chunk by chunk, thread 0 carries the chain
            const int q = q0, sp = split[q];
            double acc = b[lo + q];
            for (int base = k0; base < k1; base += kTileEntries) {
                const int m = min(kTileEntries, k1 - base);
                stage_any(sm.v, base, base + m, M.ci, M.v, M.pk, M.pv, M.pb, bq, q0, (double *)nullptr, [&](int c) -> double { return x(c); });
                __syncthreads();
                if (M.tree_long) {   // free order: the N part and the L part of the chunk tree-summed
                    const int cut = min(max(sp - base, 0), m);
                    const double c1 = block_tree_sum(sm.v, 0, cut, sm.red);
                    const double c2 = block_tree_sum(sm.v, cut, m, sm.red);
                    if (threadIdx.x == 0) {
                        acc -= c1;
                        if (sp >= base && sp < base + m) P[q] = acc;
                        acc -= c2;
                    }
                } else if (threadIdx.x == 0) {
                    if (sp >= base && sp < base + m) {
                        acc = chain_sub(acc, sm.v, 0, sp - base);
                        P[q] = acc;
                        acc = chain_sub(acc, sm.v, sp - base, m);
                    } else {
                        acc = chain_sub(acc, sm.v, 0, m);
                    }
                }
                __syncthreads();
            }
            if (threadIdx.x == 0) {
                if (sp == k1) P[q] = acc;   // no L entries
                finish(q, acc);
            }
        }
    }
}

// Inner step over the L-only rows:  y_q = (P_q - sum_{L_i} a yp[j - lo]) / d  (keeps yp_q if |d| small)
// (column c reads ycols[c - col_off]; a row with |d| small keeps ykeep[q]; rows are lo + q)
template <int PATH>   // 0 tile, 1 wave chain, 2 wave tree (free order)
__global__ __launch_bounds__(kBlock) void ts_inner(int lo, DevCSR M, const double *__restrict__ deff,
                                                   const double *__restrict__ P, const double *ycols, int col_off,
                                                   const double *ykeep, double *__restrict__ y)
{
    auto fetch = [&](int c) -> double { return ycols[c - col_off]; };
    auto finish = [&](int q, double acc) {
        const double d = deff[lo + q];
        y[q] = fabs(d) > SMALLFLOAT ? acc / d : ykeep[q];
    };
    if constexpr (PATH >= kXell) {   // column ELL rows of width PATH - kXell: one thread per row
        constexpr int W = PATH - kXell;
        __shared__ XellSmem es;
        const int bq = blockIdx.x;
        const int2 ba = M.bk[bq], be = M.bk[bq + 1];
        const int q = ba.x + (int)threadIdx.x;
        const bool live = q < be.x;
        unsigned w[W];
        double pq = 0.0, dq = 0.0;
#pragma unroll
        for (int t = 0; t < W; ++t) w[t] = 0xffffffffu;
        if (live) {   // codes, P_q and the divisor in flight across the barrier
            xell_codes<W>(M.dv_xell, q, w);
            pq = P[q];
            dq = deff[lo + q];
        }
        {
            const int4 pq4 = M.dv_pd[bq];
            for (int t = threadIdx.x; t < pq4.w; t += kBlock) es.vd[t] = M.dv_vd[pq4.z + t];
        }
        __syncthreads();
        if (live) {
            double xv[W];
            int ds;
            const int len = xell_gather<W>(w, -1, M.xell_shift, fetch, xv, ds);
            const double acc = xell_sub(pq, w, xv, es, M.xell_shift, 0, len);
            y[q] = fabs(dq) > SMALLFLOAT ? acc / dq : ykeep[q];   // finish() with the divisor loaded early
        }
        return;
    } else if constexpr (PATH >= 3) {   // merged row groups, G = PATH, M.mg_W waves per group
        constexpr int G = PATH;
        __shared__ double red[8 * G];
        int g = 0, u = 0;
        double l_sum = 0.0, unused = 0.0;
        if (merged_block<G, 1>(M.mg_gp, M.mg_ng, M.mg_W, M.mg_k, M.mg_v, fetch,
                               red, g, u, l_sum, unused)) {
            const int q = g * G + u;
            if (q < M.n) finish(q, P[q] - l_sum);
        }
        return;
    } else if constexpr (PATH == 2) {
        const int q = xcd_bid() * 4 + (threadIdx.x >> 6);
        if (q >= M.n) return;
        const double acc =
            P[q] - wave_row_sum(M.rp[q], M.rp[q + 1], M.ci, M.v, [&](int c, double a) { return a * fetch(c); });
        if ((threadIdx.x & 63) == 0) finish(q, acc);
        return;
    } else if constexpr (PATH == 1) {
        __shared__ __attribute__((aligned(16))) double strips[4][kWaveStage];
        const int wave = threadIdx.x >> 6, q = xcd_bid() * 4 + wave;
        if (q >= M.n) return;
        const double acc = wave_row_chain<true>(
            M.rp[q], M.rp[q + 1], M.ci, M.v, [&](int c, double a) { return a * fetch(c); }, P[q], strips[wave]);
        if ((threadIdx.x & 63) == 0) finish(q, acc);
        return;
    } else {
        __shared__ SpmvSmem sm;
        const int bq = xcd_bid();
        const BlockBounds bb = block_bounds(M.bk, M.rp, bq);
        const int q0 = bb.r0, q1 = bb.r1, k0 = bb.k0, k1 = bb.k1;
        if (k1 - k0 <= kTileEntries) {
            const int q = q0 + (int)threadIdx.x;
            int a = 0, e = 0;
            double acc = 0.0;
            if (q < q1) a = M.rp[q] - k0, e = M.rp[q + 1] - k0, acc = P[q];
            stage_any(sm.v, k0, k1, M.ci, M.v, M.pk, M.pv, M.pb, bq, q0, (double *)nullptr, fetch);
            __syncthreads();
            if (q < q1) finish(q, chain_sub(acc, sm.v, a, e));
        } else {
            const int q = q0;
            double acc = P[q];
            for (int base = k0; base < k1; base += kTileEntries) {
                const int m = min(kTileEntries, k1 - base);
                stage_any(sm.v, base, base + m, M.ci, M.v, M.pk, M.pv, M.pb, bq, q0, (double *)nullptr, fetch);
                __syncthreads();
                if (M.tree_long) {
                    const double c = block_tree_sum(sm.v, 0, m, sm.red);
                    if (threadIdx.x == 0) acc -= c;
                } else if (threadIdx.x == 0) {
                    acc = chain_sub(acc, sm.v, 0, m);
                }
                __syncthreads();
            }
            if (threadIdx.x == 0) finish(q, acc);
        }
    }
}

// ledger (sss_engine.hpp ByteLedger): a pass's matrix bytes -- the rows [lo, hi) of a contiguous class,
// else the pass's share of A -- + the x it gathers (8 B per row) + `vec` bytes of row vectors per row
static void ledger_pass(const DevCSR &A, const PassSchedule &ps, double vec)
{
    if (!ledger_on()) return;
    const double mat = ps.range ? matrix_bytes_rows(A, ps.lo, ps.hi)
                                : (A.n ? (double)A.stream_bytes * ps.nrows / A.n : 0.0);
    ledger_add(mat + (8.0 + vec) * ps.nrows);
}

void launch_ts_stage0(const DevCSR &M, int lo, const int *split, const double *b, XSrc x, const double *deff,
                      double *P, double *y, hipStream_t s)
{
    if (M.n == 0) return;
    ledger_add((double)M.stream_bytes + 40.0 * M.n);   // + x gathers, b, deff, P and y
    if (M.mg_G == 8 && M.mg_two)
        hipLaunchKernelGGL(ts_stage0<8>, dim3(M.ngrid), dim3(kBlock), 0, s, lo, M, split, b, x, deff, P, y);
    else if (M.mg_G == 4 && M.mg_two)
        hipLaunchKernelGGL(ts_stage0<4>, dim3(M.ngrid), dim3(kBlock), 0, s, lo, M, split, b, x, deff, P, y);
    else if (M.vec_rows)
        hipLaunchKernelGGL(ts_stage0<2>, dim3((M.n + 3) / 4), dim3(kBlock), 0, s, lo, M, split, b, x, deff, P, y);
    else if (M.wave_rows)
        hipLaunchKernelGGL(ts_stage0<1>, dim3(M.ngrid), dim3(kBlock), 0, s, lo, M, split, b, x, deff, P, y);
    else if (M.dv_xell)
        with_tile_kind(M, [&](auto K) {
            constexpr int KK = decltype(K)::value;
            if constexpr (KK >= kXell)
                hipLaunchKernelGGL(ts_stage0<KK>, dim3(M.nblk), dim3(kBlock), 0, s, lo, M, split, b, x, deff, P, y);
        });
    else
        hipLaunchKernelGGL(ts_stage0<0>, dim3(M.nblk), dim3(kBlock), 0, s, lo, M, split, b, x, deff, P, y);
}

void launch_ts_inner(const DevCSR &M, int lo, const double *deff, const double *P, const double *ycols, int col_off,
                     const double *ykeep, double *y, hipStream_t s)
{
    if (M.n == 0) return;
    ledger_add((double)M.stream_bytes + 40.0 * M.n);   // + y gathers, deff, P, ykeep and y
    if (M.mg_G == 8)
        hipLaunchKernelGGL(ts_inner<8>, dim3(M.ngrid), dim3(kBlock), 0, s, lo, M, deff, P, ycols, col_off, ykeep, y);
    else if (M.mg_G == 4)
        hipLaunchKernelGGL(ts_inner<4>, dim3(M.ngrid), dim3(kBlock), 0, s, lo, M, deff, P, ycols, col_off, ykeep, y);
    else if (M.vec_rows)
        hipLaunchKernelGGL(ts_inner<2>, dim3((M.n + 3) / 4), dim3(kBlock), 0, s, lo, M, deff, P, ycols, col_off, ykeep, y);
    else if (M.wave_rows)
        hipLaunchKernelGGL(ts_inner<1>, dim3(M.ngrid), dim3(kBlock), 0, s, lo, M, deff, P, ycols, col_off, ykeep, y);
    else if (M.dv_xell)
        with_tile_kind(M, [&](auto K) {
            constexpr int KK = decltype(K)::value;
            if constexpr (KK >= kXell)
                hipLaunchKernelGGL(ts_inner<KK>, dim3(M.nblk), dim3(kBlock), 0, s, lo, M, deff, P, ycols, col_off, ykeep,
                                   y);
        });
    else
        hipLaunchKernelGGL(ts_inner<0>, dim3(M.nblk), dim3(kBlock), 0, s, lo, M, deff, P, ycols, col_off, ykeep, y);
}

// First pass of a smoother call on a zero iterate (C/F-Jacobi pass or two-stage stage 0 right after
// the cycle zeroed x): every product a_k * x_k is +-0.0, so t = b - (a_1 x_1) - (a_2 x_2) - ... is
// exactly b -- except b == -0.0 with a summed value whose sign bit is set (its product -0.0 turns
// -0.0 into +0.0), which is order-independent.  The pass then reads no matrix entries (the rare
// -0.0 rows scan their values).  Requires finite matrix values (SmootherPlan::finite).
__device__ __forceinline__ double zero_x_sum(double t, const int *__restrict__ ci, const double *__restrict__ v, int a,
                                             int e, int skip_col)
{
    if (t == 0.0 && signbit(t))
        for (int k = a; k < e; ++k)
            if (ci[k] != skip_col && signbit(v[k])) return 0.0;
    return t;
}

template <bool TWO>
__global__ __launch_bounds__(kBlock) void zero_first_pass(int lo, int m, const int *__restrict__ rp,
                                                          const int *__restrict__ ci, const double *__restrict__ v,
                                                          const int *__restrict__ split, const double *__restrict__ b,
                                                          const double *__restrict__ deff, double *__restrict__ P,
                                                          double *__restrict__ y)
{
    const int q = blockIdx.x * kBlock + threadIdx.x;
    if (q >= m) return;
    const int r = lo + q;
    double t;
    if (TWO) {   // rows of the pass's [N | L] matrix (local numbering): P = b - N x, t = P - L x
        const double Pq = zero_x_sum(b[r], ci, v, rp[q], split[q], -1);
        P[q] = Pq;
        t = zero_x_sum(Pq, ci, v, split[q], rp[q + 1], -1);
    } else {     // rows of the level matrix: every entry but the diagonal
        t = zero_x_sum(b[r], ci, v, rp[r], rp[r + 1], r);
    }
    const double d = deff[r];
    y[q] = fabs(d) > SMALLFLOAT ? t / d : 0.0;   // a row that keeps its value keeps x_r = +0.0
}

int launch_f_residual_pending(const SmootherPlan &sp, const DevCSR &A, const double *b, const double *x, double *r,
                              double *partial, double *pend, hipStream_t s)
{
    if (!sp.pend_ok) return ERROR_INPUT_PAR;
    const PassSchedule &F = sp.pass[0];
    const double *deff = (sp.own_diag && (A.pk || has_dict(A))) ? nullptr : sp.d_first;
    ledger_pass(A, F, deff ? 40.0 : 32.0);   // b, r, pend (and deff)
    with_tile_kind(A, [&](auto K) {
        launch_relax_range<3, decltype(K)::value>(F.blo, F.bhi - F.blo, s, devdict(A, 0), A.bk, A.rp, A.ci, A.v,
                                                  sp.diag_pos, F.lo, b, const_cast<double *>(x), (const double *)nullptr,
                                                  pend, deff, A.pk, A.pv, A.pb, r, partial, xsrc_of(x));
    });
    SSS_HIP(hipGetLastError());
    return 0;
}

__global__ __launch_bounds__(kBlock) void scatter_rows(int m, const int *__restrict__ map, const double *__restrict__ y,
                                                       double *__restrict__ x)
{
    const int r = blockIdx.x * kBlock + threadIdx.x;
    if (r < m) x[map[r]] = y[r];
}

// One launch per DAG depth of an exact pass (the schedule of PassSchedule::h_off).
static int depth_launches(const PassSchedule &ps, bool long_rows, bool nat, const DevCSR &A, const double *b, double *x,
                          const double *deff, hipStream_t s)
{
    ledger_pass(A, ps, 24.0);   // b, deff, x written
    for (int l = 0; l < ps.depth; ++l) {
        const int off = ps.h_off[l], cnt = ps.h_off[l + 1] - off;
        if (cnt == 0) continue;
        if (long_rows)
            hipLaunchKernelGGL(nat ? gs_depth_wave<true> : gs_depth_wave<false>, dim3((cnt + 3) / 4), dim3(kBlock), 0, s,
                               ps.rows + off, cnt, A.rp, A.ci, A.v, b, x, deff);
        else
            hipLaunchKernelGGL(nat ? gs_depth_thread<true> : gs_depth_thread<false>, dim3((cnt + kBlock - 1) / kBlock),
                               dim3(kBlock), 0, s, ps.rows + off, cnt, A.rp, A.ci, A.v, b, x, deff);
    }
    SSS_HIP(hipGetLastError());
    return 0;
}

int smoother_build_natural(SmootherPlan &sp, const SSS_MAT &A, int lo, int hi)
{
    const int n = A.num_rows, m = hi - lo;
    const int *rp = A.row_ptr, *ci = A.col_idx;
    const double *v = A.val;
    int rc;
    sp.kind = SSS_HIP_SMOOTH_EXACT;
    sp.natural = true;
    long long nnz = 0;
    for (int i = lo; i < hi; ++i) nnz += rp[i + 1] - rp[i];
    sp.long_rows = m > 0 && nnz >= (long long)std::min(32, wave_row_min()) * m;
    // the carried reciprocal d (Solve/SSS_smooth.c:106-109): per direction, first sweep from
    // d = 0, later sweeps from the previous sweep's last value
    std::vector<double> df[2] = {std::vector<double>(n, 0.0), std::vector<double>(n, 0.0)},
                        dl[2] = {std::vector<double>(n, 0.0), std::vector<double>(n, 0.0)};
    for (int dir = 0; dir < 2; ++dir) {
        double d = 0.0;
        for (int sweep = 0; sweep < 2; ++sweep)
            for (int q = 0; q < m; ++q) {
                const int i = dir == 0 ? lo + q : hi - 1 - q;
                for (int k = rp[i]; k < rp[i + 1]; ++k)
                    if (ci[k] == i && SSS_ABS(v[k]) > SMALLFLOAT) d = 1.e+0 / v[k];
                (sweep == 0 ? df : dl)[dir][i] = d;
            }
    }
    // level schedules: ascending (row i reads the new x_j of coupled j < i, the old x_j of j > i,
    // which must wait for it) and descending (mirrored)
    for (int dir = 0; dir < 2; ++dir) {
        PassSchedule &ps = sp.pass[dir];
        std::vector<int> depth(n, 0), pushed(n, 0);
        auto in = [&](int j) { return j >= lo && j < hi; };
        for (int q = 0; q < m; ++q) {
            const int i = dir == 0 ? lo + q : hi - 1 - q;
            int dep = pushed[i];
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                const int j = ci[k];
                if (in(j) && (dir == 0 ? j < i : j > i)) dep = std::max(dep, depth[j] + 1);
            }
            depth[i] = dep;
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                const int j = ci[k];
                if (in(j) && (dir == 0 ? j > i : j < i)) pushed[j] = std::max(pushed[j], dep + 1);
            }
        }
        int maxd = -1;
        for (int i = lo; i < hi; ++i) maxd = std::max(maxd, depth[i]);
        ps.depth = maxd + 1;
        ps.h_off.assign(ps.depth + 1, 0);
        for (int i = lo; i < hi; ++i) ps.h_off[depth[i] + 1]++;
        for (int l = 0; l < ps.depth; ++l) ps.h_off[l + 1] += ps.h_off[l];
        ps.nrows = m;
        std::vector<int> fill(ps.h_off.begin(), ps.h_off.end()), rows(std::max(m, 1));
        for (int i = lo; i < hi; ++i) rows[fill[depth[i]]++] = i;
        if ((rc = upload_ints(&ps.rows, rows))) return rc;
        if (ps.depth > 1 && (rc = gs_persist_build(ps, A, lo, hi, sp.long_rows, true, dir == 1))) return rc;
    }
    if ((rc = upload_doubles(&sp.d_first, df[0])) || (rc = upload_doubles(&sp.d_later, dl[0])) ||
        (rc = upload_doubles(&sp.nd_first, df[1])) || (rc = upload_doubles(&sp.nd_later, dl[1])))
        return rc;
    return 0;
}

int smoother_run(const SmootherPlan &sp, const DevCSR &A, const double *b, double *x, int sweeps, hipStream_t s,
                 const PassHooks *hk, ResidFuse *rf, const double *pre_f, bool x_zero, bool post)
{
    if (sp.natural) {   // natural-order GS: ascending pre-smoother, descending post-smoother
        if (hk || pre_f) return ERROR_INPUT_PAR;
        if (rf) rf->done = false;
        const PassSchedule &ps = sp.pass[post ? 1 : 0];
        if (ps.nrows == 0) return 0;
        for (int sw = 0; sw < sweeps; ++sw) {
            const double *deff = post ? (sw == 0 ? sp.nd_first : sp.nd_later) : (sw == 0 ? sp.d_first : sp.d_later);
            if (ps.gp.engine) ledger_pass(A, ps, 24.0);
            int rc = ps.gp.engine ? gs_persist_run(ps, A, b, x, deff, s) : depth_launches(ps, sp.long_rows, true, A, b, x, deff, s);
            if (rc) return rc;
        }
        return 0;
    }
    if (rf) rf->done = false;
    if (pre_f && (!sp.pend_ok || hk || sweeps < 1)) return ERROR_INPUT_PAR;
    if (sp.fz.engine && sweeps == sp.fz.sweeps && !hk && !pre_f) {
        for (int sw = 0; sw < sweeps; ++sw)
            for (const auto &ps : sp.pass) ledger_pass(A, ps, 24.0);
        return gs_fused_run(sp.fz, A, b, x, sp.d_first, sp.d_later, x_zero, s);
    }
    const int n = A.n;
    if (n == 0) return 0;
    int rc;
    // no-copy C/F-Jacobi: where each class's current values live (x or sp.x2)
    const bool nocopy = sp.x2 && !hk;
    double *cur[2] = {x, x};
    for (int sw = 0; sw < sweeps; ++sw) {
        const double *deff = sw == 0 ? sp.d_first : sp.d_later;
        for (int c = 0; c < 2; ++c) {
            const PassSchedule &ps = sp.pass[c];
            if (ps.nrows == 0) continue;
            if (pre_f && sw == 0 && c == 0) continue;   // computed with the last residual (pre_f)
            // first pass on a just-zeroed iterate (C/F-Jacobi / two-stage): t = b, no matrix read
            const bool zfirst = x_zero && sw == 0 && c == 0 && sp.finite && sp.kind == SSS_HIP_SMOOTH_JACOBI;
            // a plain tile-path relaxation pass (exact depth-1 GS-CF, or C/F-Jacobi) can overlap the
            // halo with its interior blocks (PassHooks::split)
            const bool fused_pass = rf && sp.fuse_resid && c == 1 && sw + 1 == sweeps;
            const bool split_pass = hk && hk->split && !zfirst && !(A.wave_rows || A.vec_rows) && ps.range &&
                                    (sp.kind != SSS_HIP_SMOOTH_JACOBI || sp.inner == 0) && !nocopy;
            if (hk) {   // distributed level: refresh x's ghosts; only contiguous passes qualify
                if (!ps.range) return ERROR_INPUT_PAR;
                // a zeroed x has zero ghosts (the descent clears own rows and ghosts); `finite` is
                // agreed over the ranks, so every rank skips this exchange together
                if (!zfirst && !split_pass && (rc = hk->exchange(hk->ctx, x))) return rc;
            }
            if (ps.range) {
                const int nb = ps.bhi - ps.blo, m = ps.hi - ps.lo, nw = (m + 3) / 4;
                const bool wave = A.wave_rows || A.vec_rows;
                XSrc xs = nocopy ? XSrc{cur[0], cur[1], sp.csplit} : xsrc_of(x);
                if (pre_f && sw == 0) xs = XSrc{pre_f, x, sp.pass[0].hi};   // this sweep's F values
                // tile passes take each row's divisor from its staged diagonal (no deff stream)
                const bool tile_d = sp.own_diag && (A.pk != nullptr || has_dict(A));
                auto relax = [&](auto mode, const int *cols, const double *yp, double *y) -> int {
                    constexpr int M = decltype(mode)::value;
                    ledger_pass(A, ps, (tile_d && !wave) ? 16.0 : 24.0);   // b, the written row (and deff)
                    if (wave && A.vec_rows)
                        hipLaunchKernelGGL((relax_range_wave<M, true>), dim3(nw), dim3(kBlock), 0, s, ps.lo, ps.hi,
                                           A.rp, cols, A.v, b, x, yp, y, deff, xs);
                    else if (wave)
                        hipLaunchKernelGGL((relax_range_wave<M, false>), dim3(nw), dim3(kBlock), 0, s, ps.lo, ps.hi,
                                           A.rp, cols, A.v, b, x, yp, y, deff, xs);
                    else {
                        auto go = [&](int b0, int b1) {
                            with_tile_kind(A, [&](auto K) {
                                launch_relax_range<M, decltype(K)::value>(
                                    b0, b1 - b0, s, devdict(A, 0), A.bk, A.rp, cols, A.v, sp.diag_pos, ps.lo, b, x, yp,
                                    y, tile_d ? nullptr : deff, A.pk, A.pv, A.pb, (double *)nullptr, (double *)nullptr,
                                    xs);
                            });
                        };
                        if (split_pass) return hk->split(x, ps.blo, ps.bhi, go);
                        go(ps.blo, ps.bhi);
                    }
                    return 0;
                };
                (void)nb;
                if (sp.kind == SSS_HIP_SMOOTH_JACOBI && sp.inner > 0 && hk) {
                    // iterates live in full-length work vectors whose ghosts (lower-rank rows of
                    // this class) are refreshed after every stage
                    const DevCSR &Mn = ps.ts_nl, &Ml = ps.ts_lo;
                    double *wcur = hk->w0, *wnxt = hk->w1;
                    if (zfirst) {
                        ledger_add(32.0 * m);
                        hipLaunchKernelGGL(zero_first_pass<true>, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                                           ps.lo, m, Mn.rp, Mn.ci, Mn.v, ps.ts_split, b, deff, ps.ts_P, wcur + ps.lo);
                    } else
                        launch_ts_stage0(Mn, ps.lo, ps.ts_split, b, xsrc_of(x), deff, ps.ts_P, wcur + ps.lo, s);
                    for (int st = 0; st < sp.inner; ++st) {
                        if ((rc = hk->exchange(hk->ctx, wcur))) return rc;
                        launch_ts_inner(Ml, ps.lo, deff, ps.ts_P, wcur, 0, wcur + ps.lo, wnxt + ps.lo, s);
                        std::swap(wcur, wnxt);
                    }
                    ledger_add(16.0 * m);
                    SSS_HIP(hipMemcpyAsync(x + ps.lo, wcur + ps.lo, sizeof(double) * (size_t)m, hipMemcpyDeviceToDevice,
                                           s));
                } else if (sp.kind == SSS_HIP_SMOOTH_JACOBI && nocopy) {
                    // stage 0 (or the Jacobi pass) writes the other buffer; inner steps read only this
                    // class's previous iterate, so they alternate between the two buffers in place
                    double *prev = cur[c] == x ? sp.x2 : x, *next = cur[c];
                    const int zg = (m + kBlock - 1) / kBlock;
                    if (zfirst) ledger_add((sp.inner > 0 ? 32.0 : 24.0) * m);   // b, deff, y (and P)
                    if (zfirst && sp.inner > 0)
                        hipLaunchKernelGGL(zero_first_pass<true>, dim3(zg), dim3(kBlock), 0, s, ps.lo, m, ps.ts_nl.rp,
                                           ps.ts_nl.ci, ps.ts_nl.v, ps.ts_split, b, deff, ps.ts_P, prev + ps.lo);
                    else if (zfirst)
                        hipLaunchKernelGGL(zero_first_pass<false>, dim3(zg), dim3(kBlock), 0, s, ps.lo, m, A.rp, A.ci,
                                           A.v, (const int *)nullptr, b, deff, (double *)nullptr, prev + ps.lo);
                    else if (sp.inner > 0)
                        launch_ts_stage0(ps.ts_nl, ps.lo, ps.ts_split, b, xs, deff, ps.ts_P, prev + ps.lo, s);
                    else if ((rc = relax(std::integral_constant<int, 1>(), A.ci, (const double *)nullptr, prev + ps.lo)))
                        return rc;
                    for (int st = 0; st < sp.inner; ++st) {
                        launch_ts_inner(ps.ts_lo, ps.lo, deff, ps.ts_P, prev, 0, prev + ps.lo, next + ps.lo, s);
                        std::swap(prev, next);
                    }
                    cur[c] = prev;
                } else if (sp.kind == SSS_HIP_SMOOTH_JACOBI && sp.inner > 0) {
                    const DevCSR &Mn = ps.ts_nl, &Ml = ps.ts_lo;
                    launch_ts_stage0(Mn, ps.lo, ps.ts_split, b, xsrc_of(x), deff, ps.ts_P, ps.y, s);
                    double *ycur = ps.y, *ynxt = ps.y2;
                    for (int st = 0; st < sp.inner; ++st) {
                        launch_ts_inner(Ml, ps.lo, deff, ps.ts_P, ycur, ps.lo, ycur, ynxt, s);
                        std::swap(ycur, ynxt);
                    }
                    ledger_add(16.0 * m);
                    SSS_HIP(hipMemcpyAsync(x + ps.lo, ycur, sizeof(double) * (size_t)m, hipMemcpyDeviceToDevice, s));
                } else if (sp.kind == SSS_HIP_SMOOTH_JACOBI && zfirst) {
                    // the pass reads no x at all, so it may write x in place
                    ledger_add(24.0 * m);
                    hipLaunchKernelGGL(zero_first_pass<false>, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                                       ps.lo, m, A.rp, A.ci, A.v, (const int *)nullptr, b, deff, (double *)nullptr,
                                       x + ps.lo);
                } else if (sp.kind == SSS_HIP_SMOOTH_JACOBI) {
                    if ((rc = relax(std::integral_constant<int, 1>(), A.ci, (const double *)nullptr, ps.y))) return rc;
                    ledger_add(16.0 * m);
                    SSS_HIP(hipMemcpyAsync(x + ps.lo, ps.y, sizeof(double) * (size_t)m, hipMemcpyDeviceToDevice, s));
                } else if (fused_pass) {
                    ledger_pass(A, ps, tile_d ? 24.0 : 32.0);   // b, x and r written (and deff)
                    auto go = [&](int b0, int b1) {
                        with_tile_kind(A, [&](auto K) {
                            launch_relax_range<2, decltype(K)::value>(
                                b0, b1 - b0, s, devdict(A, 0), A.bk, A.rp, A.ci, A.v, sp.diag_pos, ps.lo, b, x,
                                (const double *)nullptr, (double *)nullptr, tile_d ? nullptr : deff, A.pk, A.pv, A.pb,
                                rf->r, rf->partial, xs);
                        });
                    };
                    if (split_pass) {
                        if ((rc = hk->split(x, ps.blo, ps.bhi, go))) return rc;
                    } else {
                        go(ps.blo, ps.bhi);
                    }
                    rf->done = true;
                } else if ((rc = relax(std::integral_constant<int, 0>(), A.ci, (const double *)nullptr, (double *)nullptr))) {
                    return rc;
                }
                if (pre_f && sw == 0 && c == 1 && sweeps == 1) {   // no later F pass overwrites x_F
                    ledger_add(16.0 * sp.pass[0].hi);
                    SSS_HIP(hipMemcpyAsync(x, pre_f, sizeof(double) * (size_t)sp.pass[0].hi, hipMemcpyDeviceToDevice, s));
                }
                continue;
            }
            if (sp.kind == SSS_HIP_SMOOTH_JACOBI) {
                ledger_add((double)ps.sub.stream_bytes + (8.0 + 24.0 + 20.0) * ps.nrows);   // + the scatter
                if (ps.sub.wave_rows)
                    hipLaunchKernelGGL(relax_wave<false>, dim3(ps.sub.ngrid), dim3(kBlock), 0, s, ps.nrows, ps.sub.rp,
                                       ps.sub.ci, ps.sub.v, ps.map, b, x, ps.y, sp.d_first);
                else
                    hipLaunchKernelGGL(relax_compact<false>, dim3(ps.sub.nblk), dim3(kBlock), 0, s, ps.sub.blk,
                                       ps.sub.rp, ps.sub.ci, ps.sub.v, ps.map, b, x, ps.y, sp.d_first);
                hipLaunchKernelGGL(scatter_rows, dim3((ps.nrows + kBlock - 1) / kBlock), dim3(kBlock), 0, s, ps.nrows,
                                   ps.map, ps.y, x);
                continue;
            }
            if (ps.compact) {
                ledger_add((double)ps.sub.stream_bytes + (8.0 + 24.0 + 4.0) * ps.nrows);   // + the row map
                if (ps.sub.wave_rows)
                    hipLaunchKernelGGL(relax_wave<true>, dim3(ps.sub.ngrid), dim3(kBlock), 0, s, ps.nrows, ps.sub.rp,
                                       ps.sub.ci, ps.sub.v, ps.map, b, x, (double *)nullptr, deff);
                else
                    hipLaunchKernelGGL(relax_compact<true>, dim3(ps.sub.nblk), dim3(kBlock), 0, s, ps.sub.blk,
                                       ps.sub.rp, ps.sub.ci, ps.sub.v, ps.map, b, x, (double *)nullptr, deff);
                continue;
            }
            if (ps.gp.engine) {
                ledger_pass(A, ps, 24.0);
                if ((rc = gs_persist_run(ps, A, b, x, deff, s))) return rc;
                continue;
            }
            if ((rc = depth_launches(ps, sp.long_rows, false, A, b, x, deff, s))) return rc;
        }
    }
    for (int c = 0; c < 2; ++c)   // odd number of writes to a class (odd sweeps x (1 + inner))
        if (cur[c] != x) {
            ledger_add(16.0 * (sp.pass[c].hi - sp.pass[c].lo));
            SSS_HIP(hipMemcpyAsync(x + sp.pass[c].lo, cur[c] + sp.pass[c].lo,
                                   sizeof(double) * (size_t)(sp.pass[c].hi - sp.pass[c].lo), hipMemcpyDeviceToDevice, s));
        }
    SSS_HIP(hipGetLastError());
    return 0;
}

}  // namespace sss
