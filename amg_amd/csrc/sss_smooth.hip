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

#include <algorithm>
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

int smoother_build(SmootherPlan &sp, const SSS_MAT &A, const int *mark, int kind)
{
    const int n = A.num_rows;
    const int *rp = A.row_ptr, *ci = A.col_idx;
    const double *v = A.val;
    std::vector<int> cls(n), depth(n, 0), pushed(n, 0);
    std::vector<double> last_diag(n, 0.0), d_first(n, 0.0), d_later(n, 0.0);
    std::vector<char> has_diag(n, 0);
    bool all_diag = true;
    int rc;

    sp.kind = kind;
    for (int i = 0; i < n; ++i) {
        cls[i] = mark ? (mark[i] == 1 ? 1 : 0) : 0;
        for (int k = rp[i]; k < rp[i + 1]; ++k)
            if (ci[k] == i) { last_diag[i] = v[k]; has_diag[i] = 1; }
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
    sp.long_rows = n > 0 && nnz_total / n > 16;
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
    }
    if ((rc = upload_ints(&sp.cls, cls))) return rc;
    if (kind == SSS_HIP_SMOOTH_JACOBI) {
        if ((rc = upload_doubles(&sp.d_first, last_diag))) return rc;   // Jacobi: row's own diagonal
        sp.d_later = sp.d_first;
        sp.x_tmp = dev_alloc<double>((size_t)n);
        if (!sp.x_tmp) return hip_fail(hipErrorOutOfMemory, "hipMalloc(x_tmp)", __FILE__, __LINE__);
    } else {
        if ((rc = upload_doubles(&sp.d_first, d_first))) return rc;
        if (all_diag) sp.d_later = sp.d_first;
        else if ((rc = upload_doubles(&sp.d_later, d_later))) return rc;
    }
    return 0;
}

void smoother_free(SmootherPlan &sp)
{
    for (auto &ps : sp.pass) dev_free(ps.rows);
    if (sp.d_later != sp.d_first) dev_free(sp.d_later);
    dev_free(sp.d_first);
    dev_free(sp.cls);
    dev_free(sp.x_tmp);
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

// exact GS, one wave per row: lanes form the products, lane 0 subtracts them in CSR order
// (the diagonal contributes +0.0, an exact identity for subtraction)
__global__ __launch_bounds__(64) void gs_depth_wave(const int *__restrict__ rows, const int *__restrict__ rp,
                                                    const int *__restrict__ ci, const double *__restrict__ v,
                                                    const double *__restrict__ b, double *x,
                                                    const double *__restrict__ deff)
{
    __shared__ double prod[64];
    const int i = rows[blockIdx.x];
    const int lane = threadIdx.x;
    const int k0 = rp[i], k1 = rp[i + 1];
    double acc = b[i];
    for (int base = k0; base < k1; base += 64) {
        const int k = base + lane;
        double p = 0.0;
        if (k < k1) {
            const int j = ci[k];
            if (j != i) p = v[k] * x[j];
        }
        prod[lane] = p;
        __syncthreads();
        if (lane == 0) {
            const int m = min(64, k1 - base);
            for (int q = 0; q < m; ++q) acc -= prod[q];
        }
        __syncthreads();
    }
    if (lane == 0) {
        const double d = deff[i];
        if (fabs(d) > SMALLFLOAT) x[i] = acc / d;
    }
}

// C/F-Jacobi pass over all rows: rows of class `c` are relaxed from x_in, others copied
__global__ __launch_bounds__(kBlock) void jacobi_pass_thread(int n, int c, const int *__restrict__ cls,
                                                             const int *__restrict__ rp, const int *__restrict__ ci,
                                                             const double *__restrict__ v, const double *__restrict__ b,
                                                             const double *__restrict__ x_in, double *__restrict__ x_out,
                                                             const double *__restrict__ dg)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    double out = x_in[i];
    if (c < 0 || cls[i] == c) {
        double acc = b[i];
        for (int k = rp[i]; k < rp[i + 1]; ++k) {
            const int j = ci[k];
            if (j != i) acc -= v[k] * x_in[j];
        }
        const double d = dg[i];
        if (fabs(d) > SMALLFLOAT) out = acc / d;
    }
    x_out[i] = out;
}

__global__ __launch_bounds__(64) void jacobi_pass_wave(int c, const int *__restrict__ cls, const int *__restrict__ rp,
                                                       const int *__restrict__ ci, const double *__restrict__ v,
                                                       const double *__restrict__ b, const double *__restrict__ x_in,
                                                       double *__restrict__ x_out, const double *__restrict__ dg)
{
    __shared__ double prod[64];
    const int i = blockIdx.x;
    const int lane = threadIdx.x;
    if (!(c < 0 || cls[i] == c)) {
        if (lane == 0) x_out[i] = x_in[i];
        return;
    }
    const int k0 = rp[i], k1 = rp[i + 1];
    double acc = b[i];
    for (int base = k0; base < k1; base += 64) {
        const int k = base + lane;
        double p = 0.0;
        if (k < k1) {
            const int j = ci[k];
            if (j != i) p = v[k] * x_in[j];
        }
        prod[lane] = p;
        __syncthreads();
        if (lane == 0) {
            const int m = min(64, k1 - base);
            for (int q = 0; q < m; ++q) acc -= prod[q];
        }
        __syncthreads();
    }
    if (lane == 0) {
        const double d = dg[i];
        x_out[i] = fabs(d) > SMALLFLOAT ? acc / d : x_in[i];
    }
}

int smoother_run(const SmootherPlan &sp, const DevCSR &A, const double *b, double *x, int sweeps, hipStream_t s)
{
    const int n = A.n;
    if (n == 0) return 0;
    if (sp.kind == SSS_HIP_SMOOTH_JACOBI) {
        double *cur = x, *nxt = sp.x_tmp;
        for (int sw = 0; sw < sweeps; ++sw) {
            for (int c = 0; c < 2; ++c) {
                if (sp.pass[c].nrows == 0) continue;
                if (sp.long_rows)
                    hipLaunchKernelGGL(jacobi_pass_wave, dim3(n), dim3(64), 0, s, c, sp.cls, A.rp, A.ci, A.v, b, cur,
                                       nxt, sp.d_first);
                else
                    hipLaunchKernelGGL(jacobi_pass_thread, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, n, c,
                                       sp.cls, A.rp, A.ci, A.v, b, cur, nxt, sp.d_first);
                std::swap(cur, nxt);
            }
        }
        if (cur != x) SSS_HIP(hipMemcpyAsync(x, cur, sizeof(double) * (size_t)n, hipMemcpyDeviceToDevice, s));
        SSS_HIP(hipGetLastError());
        return 0;
    }
    for (int sw = 0; sw < sweeps; ++sw) {
        const double *deff = sw == 0 ? sp.d_first : sp.d_later;
        for (int c = 0; c < 2; ++c) {
            const PassSchedule &ps = sp.pass[c];
            for (int l = 0; l < ps.depth; ++l) {
                const int off = ps.h_off[l], cnt = ps.h_off[l + 1] - off;
                if (cnt == 0) continue;
                if (sp.long_rows)
                    hipLaunchKernelGGL(gs_depth_wave, dim3(cnt), dim3(64), 0, s, ps.rows + off, A.rp, A.ci, A.v, b, x,
                                       deff);
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
