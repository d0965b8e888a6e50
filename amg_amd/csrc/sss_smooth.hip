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
#include <type_traits>
#include <cmath>

namespace sss {

// ---- host-side planning ---------------------------------------------------------------------
static int upload_ints(int **dst, const std::vector<int> &src)
{
    *dst = dev_alloc<int>(src.size());
    if (!*dst) return hip_fail(hipErrorOutOfMemory, "hipMalloc(ints)", __FILE__, __LINE__);
    if (!src.empty()) SSS_HIP(hipMemcpy(*dst, src.data(), sizeof(int) * src.size(), hipMemcpyHostToDevice));
    return 0;
}
static int upload_doubles(double **dst, const std::vector<double> &src)
{
    *dst = dev_alloc<double>(src.size());
    if (!*dst) return hip_fail(hipErrorOutOfMemory, "hipMalloc(doubles)", __FILE__, __LINE__);
    if (!src.empty()) SSS_HIP(hipMemcpy(*dst, src.data(), sizeof(double) * src.size(), hipMemcpyHostToDevice));
    return 0;
}

int smoother_build(SmootherPlan &sp, const SSS_MAT &A, const int *mark, int kind, const DevCSR *dA, int inner)
{
    const int n = A.num_rows;
    const int *rp = A.row_ptr, *ci = A.col_idx;
    const double *v = A.val;
    std::vector<int> cls(n), depth(n, 0), pushed(n, 0);
    std::vector<double> last_diag(n, 0.0), d_first(n, 0.0), d_later(n, 0.0);
    std::vector<char> has_diag(n, 0);
    std::vector<int> diag_pos(n, -1);
    bool all_diag = true, single_diag = true;
    int rc;

    sp.kind = kind;
    for (int i = 0; i < n; ++i) {
        cls[i] = mark ? (mark[i] == 1 ? 1 : 0) : 0;
        for (int k = rp[i]; k < rp[i + 1]; ++k)
            if (ci[k] == i) {
                last_diag[i] = v[k];
                if (has_diag[i]) single_diag = false;
                has_diag[i] = 1;
                diag_pos[i] = k;
            }
        all_diag = all_diag && has_diag[i];
    }
    // stale-d resolution: simulate the divisor register over two sweeps of (F pass, C pass)
    {
        double d = 0.0;
        for (int sweep = 0; sweep < 2; ++sweep)
            for (int c = 0; c < 2; ++c)
                for (int i = 0; i < n; ++i) {
                    if (cls[i] != c) continue;
                    if (has_diag[i]) d = last_diag[i];
                    (sweep == 0 ? d_first : d_later)[i] = d;
                }
    }
    // level schedule per class
    long long nnz_total = rp[n];
    // exact GS depth launches hold few rows each: a wave per row pays from short lengths on
    sp.long_rows = n > 0 && nnz_total >= (long long)std::min(32, wave_row_min()) * n;
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
    if (kind == SSS_HIP_SMOOTH_JACOBI && inner > 0 && sp.pass[0].range == (sp.pass[0].nrows > 0) &&
        sp.pass[1].range == (sp.pass[1].nrows > 0)) {
        // two-stage: mark same-class strictly-lower entries (j < i) as ~j in a private column copy
        sp.inner = inner;
        std::vector<int> cts(ci, ci + rp[n]);
        for (int i = 0; i < n; ++i)
            for (int k = rp[i]; k < rp[i + 1]; ++k)
                if (ci[k] < i && cls[ci[k]] == cls[i]) cts[k] = ~ci[k];
        if ((rc = upload_ints(&sp.cts, cts))) return rc;
    }
    if (sp.pass[0].range || sp.pass[1].range)
        if ((rc = upload_ints(&sp.diag_pos, diag_pos))) return rc;
    if (kind == SSS_HIP_SMOOTH_JACOBI) {
        if ((rc = upload_doubles(&sp.d_first, last_diag))) return rc;   // Jacobi: row's own diagonal
        sp.d_later = sp.d_first;
    } else {
        if ((rc = upload_doubles(&sp.d_first, d_first))) return rc;
        if (all_diag) sp.d_later = sp.d_first;
        else if ((rc = upload_doubles(&sp.d_later, d_later))) return rc;
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
    }
    if (sp.d_later != sp.d_first) dev_free(sp.d_later);
    dev_free(sp.d_first);
    dev_free(sp.cls);
    dev_free(sp.diag_pos);
    dev_free(sp.cts);
    sp = SmootherPlan();
}

// ---- kernels -------------------------------------------------------------------------------
// exact GS, one thread per row of the current depth
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
    if (fabs(d) > SMALLFLOAT) x[i] = acc / d;
}

// exact GS on long rows: four rows of the current depth per workgroup, one per wave; lanes
// gather the products, lane 0 subtracts them in CSR order (sss_spmv_dev.hpp wave_row_chain).
__global__ __launch_bounds__(kBlock) void gs_depth_wave(const int *__restrict__ rows, int cnt,
                                                        const int *__restrict__ rp, const int *__restrict__ ci,
                                                        const double *__restrict__ v, const double *__restrict__ b,
                                                        double *x, const double *__restrict__ deff)
{
    __shared__ double strips[4][kWaveStage];
    const int wave = threadIdx.x >> 6;
    const int t = blockIdx.x * 4 + wave;
    if (t >= cnt) return;
    const int i = rows[t];
    const double acc = wave_row_chain<true>(
        rp[i], rp[i + 1], ci, v, [&](int c, double a) { return c == i ? 0.0 : a * x[c]; }, b[i], strips[wave]);
    if ((threadIdx.x & 63) == 0) {
        const double d = deff[i];
        if (fabs(d) > SMALLFLOAT) x[i] = acc / d;
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
    __shared__ double strips[4][kWaveStage];
    const int wave = threadIdx.x >> 6;
    const int r = blockIdx.x * 4 + wave;
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
//   MODE 2: two-stage inner step: same-class strictly-lower entries (encoded ~j in `ci`) read the
//           previous inner iterate yp[j - lo], every other entry x[j] (from before the pass).
// t = b_r - sum over off-diagonal entries in stored order (diag_pos skips the diagonal); rows with
// |d| <= 1e-20 keep their value.  Columns may carry the two-stage encoding in every mode.
template <int MODE>
__global__ __launch_bounds__(kBlock) void relax_range(int blo, const int *__restrict__ blk, const int *__restrict__ rp,
                                                      const int *__restrict__ ci, const double *__restrict__ v,
                                                      const int *__restrict__ diag_pos, int lo,
                                                      const double *__restrict__ b, double *x,
                                                      const double *__restrict__ yp, double *__restrict__ y,
                                                      const double *__restrict__ deff)
{
    __shared__ SpmvSmem sm;
    const int bid = blo + blockIdx.x;
    const int r0 = blk[bid], r1 = blk[bid + 1];
    const int k0 = rp[r0], k1 = rp[r1];
    auto fetch = [&](int c) -> double {
        if (MODE == 2) return c < 0 ? yp[~c - lo] : x[c];
        return x[c < 0 ? ~c : c];
    };
    auto finish = [&](int r, double acc) {
        const double d = deff[r];
        if (MODE == 0) {
            if (fabs(d) > SMALLFLOAT) x[r] = acc / d;
        } else {
            const double keep = MODE == 2 ? yp[r - lo] : x[r];
            y[r - lo] = fabs(d) > SMALLFLOAT ? acc / d : keep;
        }
    };
    if (k1 - k0 <= kTileEntries) {
        const int r = r0 + (int)threadIdx.x;
        int a = 0, e = 0, dp = -1;
        double acc = 0.0;
        if (r < r1) a = rp[r] - k0, e = rp[r + 1] - k0, dp = diag_pos[r], acc = b[r];   // ahead of the tile
        stage_products_f(sm.v, k0, k1, ci, v, fetch);
        __syncthreads();
        if (r < r1) {
            if (dp < 0) acc = chain_sub(acc, sm.v, a, e);
            else {
                acc = chain_sub(acc, sm.v, a, dp - k0);
                acc = chain_sub(acc, sm.v, dp - k0 + 1, e);
            }
            finish(r, acc);
        }
    } else {
        const int r = r0, dp = diag_pos[r];
        double acc = b[r];
        for (int base = k0; base < k1; base += kTileEntries) {
            const int m = min(kTileEntries, k1 - base);
            stage_products_f(sm.v, base, base + m, ci, v, fetch);
            __syncthreads();
            if (threadIdx.x == 0) {
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

// relax_range for long-row levels: one wave per row (rows lo + 4 * blockIdx.x + wave).  The
// diagonal (single per row on range levels) contributes an exact 0.0 to the chain.
template <int MODE>
__global__ __launch_bounds__(kBlock) void relax_range_wave(int lo, int hi, const int *__restrict__ rp,
                                                           const int *__restrict__ ci, const double *__restrict__ v,
                                                           const double *__restrict__ b, double *x,
                                                           const double *__restrict__ yp, double *__restrict__ y,
                                                           const double *__restrict__ deff)
{
    __shared__ double strips[4][kWaveStage];
    const int wave = threadIdx.x >> 6;
    const int r = lo + blockIdx.x * 4 + wave;
    if (r >= hi) return;
    const double acc = wave_row_chain<true>(
        rp[r], rp[r + 1], ci, v,
        [&](int c, double a) -> double {
            if (c == r) return 0.0;
            if (MODE == 2) return a * (c < 0 ? yp[~c - lo] : x[c]);
            return a * x[c < 0 ? ~c : c];
        },
        b[r], strips[wave]);
    if ((threadIdx.x & 63) == 0) {
        const double d = deff[r];
        if (MODE == 0) {
            if (fabs(d) > SMALLFLOAT) x[r] = acc / d;
        } else {
            const double keep = MODE == 2 ? yp[r - lo] : x[r];
            y[r - lo] = fabs(d) > SMALLFLOAT ? acc / d : keep;
        }
    }
}

__global__ __launch_bounds__(kBlock) void scatter_rows(int m, const int *__restrict__ map, const double *__restrict__ y,
                                                       double *__restrict__ x)
{
    const int r = blockIdx.x * kBlock + threadIdx.x;
    if (r < m) x[map[r]] = y[r];
}

int smoother_run(const SmootherPlan &sp, const DevCSR &A, const double *b, double *x, int sweeps, hipStream_t s)
{
    const int n = A.n;
    if (n == 0) return 0;
    for (int sw = 0; sw < sweeps; ++sw) {
        const double *deff = sw == 0 ? sp.d_first : sp.d_later;
        for (int c = 0; c < 2; ++c) {
            const PassSchedule &ps = sp.pass[c];
            if (ps.nrows == 0) continue;
            if (ps.range) {
                const int nb = ps.bhi - ps.blo, m = ps.hi - ps.lo, nw = (m + 3) / 4;
                const bool wave = A.wave_rows;
                auto relax = [&](auto mode, const int *cols, const double *yp, double *y) {
                    constexpr int M = decltype(mode)::value;
                    if (wave)
                        hipLaunchKernelGGL(relax_range_wave<M>, dim3(nw), dim3(kBlock), 0, s, ps.lo, ps.hi, A.rp, cols,
                                           A.v, b, x, yp, y, deff);
                    else
                        hipLaunchKernelGGL(relax_range<M>, dim3(nb), dim3(kBlock), 0, s, ps.blo, A.blk, A.rp, cols,
                                           A.v, sp.diag_pos, ps.lo, b, x, yp, y, deff);
                };
                if (sp.kind == SSS_HIP_SMOOTH_JACOBI) {
                    const int *cols = sp.cts ? sp.cts : A.ci;
                    relax(std::integral_constant<int, 1>(), cols, (const double *)nullptr, ps.y);
                    double *cur = ps.y, *nxt = ps.y2;
                    for (int st = 0; st < sp.inner; ++st) {
                        relax(std::integral_constant<int, 2>(), cols, (const double *)cur, nxt);
                        std::swap(cur, nxt);
                    }
                    SSS_HIP(hipMemcpyAsync(x + ps.lo, cur, sizeof(double) * (size_t)m, hipMemcpyDeviceToDevice, s));
                } else {
                    relax(std::integral_constant<int, 0>(), A.ci, (const double *)nullptr, (double *)nullptr);
                }
                continue;
            }
            if (sp.kind == SSS_HIP_SMOOTH_JACOBI) {
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
                if (ps.sub.wave_rows)
                    hipLaunchKernelGGL(relax_wave<true>, dim3(ps.sub.ngrid), dim3(kBlock), 0, s, ps.nrows, ps.sub.rp,
                                       ps.sub.ci, ps.sub.v, ps.map, b, x, (double *)nullptr, deff);
                else
                    hipLaunchKernelGGL(relax_compact<true>, dim3(ps.sub.nblk), dim3(kBlock), 0, s, ps.sub.blk,
                                       ps.sub.rp, ps.sub.ci, ps.sub.v, ps.map, b, x, (double *)nullptr, deff);
                continue;
            }
            for (int l = 0; l < ps.depth; ++l) {
                const int off = ps.h_off[l], cnt = ps.h_off[l + 1] - off;
                if (cnt == 0) continue;
                if (sp.long_rows)
                    hipLaunchKernelGGL(gs_depth_wave, dim3((cnt + 3) / 4), dim3(kBlock), 0, s, ps.rows + off, cnt, A.rp,
                                       A.ci, A.v, b, x, deff);
                else
                    hipLaunchKernelGGL(gs_depth_thread, dim3((cnt + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                                       ps.rows + off, cnt, A.rp, A.ci, A.v, b, x, deff);
            }
        }
    }
    SSS_HIP(hipGetLastError());
    return 0;
}

}  // namespace sss
