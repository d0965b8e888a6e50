// sss_coarse_krylov.hip — the reference coarsest-grid solver on the GPU (parity coarse mode).
//
// SSS_amg_coarest_solve (Solve/SSS_cycle.cu:819-846) runs SSS_solver_cg (:15-437) and, if it
// fails, SSS_solver_gmres (:440-817), with the coarse SpMVs on the device (spmv_cuda /
// alpha_spmv_cuda, Solve/SSS_cuda.cu:120-165).  This file keeps the algorithm AS COMPILED
// (SURVEY.md fact 4 and Appendix A rows 5-6):
//   * CG: beta == temp1/temp1 == 1 and temp1 frozen at (r0, r0); t += A*p accumulates (t is
//     never cleared); (z, r) is computed and discarded; stagnation / false-convergence /
//     best-so-far logic exactly as written; maxit = max(250, min(n*n, 1000)).
//   * GMRES(30): Arnoldi p[i] += A*r accumulates into a vector that keeps its old content.
//   * row cap: 0 = every row (the "uncapped" parity definition); 4096 = as shipped.
// The CSR, vectors and scalars stay in HBM (the reference re-uploads the whole coarse CSR for
// every one of its ~1,000 SpMVs per V-cycle).
//
// CG control flow runs on the device: every iteration is four launches (SpMV+dot, update+
// norms, checks [+ residual re-computation when a check fires], p-update+commit).  Scalar
// decisions are recomputed identically by every workgroup from deterministic partial sums;
// workgroup 0 publishes them into a state double-buffered across iterations, so no kernel
// reads a word it (or a sibling workgroup of the same launch) writes.  The host only polls the
// stop flag every 32 iterations.  GMRES is host-steered: one 8-byte-per-entry Hessenberg
// column read back per Arnoldi step, the Givens recurrences on the host in the reference's
// exact arithmetic.
//
// Dot products / norms use fixed-order (but not sequential) reductions: results match the
// sequential host reference to ~1e-15 relative per reduction, not bitwise (tolerance ladder,
// SURVEY.md §8c).
#include "sss_engine.hpp"
#include "sss_spmv_dev.hpp"

#include <cmath>
#include <cstring>
#include <vector>

namespace sss {

enum { CG_RUN = 0, CG_STOP = 1 };
constexpr int kPoll = 32;

struct CgState {
    int mode, iter, iter_best, stag, more_step, skip_restore;
    double absres, absres0, absres_best, relres;
};
struct CgConst {
    double temp1, normr0, tol, maxdiff;
    int maxit, status;
};
struct CgMailB {
    double alpha;
    int breakdown;
};
struct CgMailC {
    double absres, relres;
    int copy_best, solstag, stag_fire, conv_check;
};

struct CoarseKrylov {
    int n = 0, cap = 0, nbe = 0, nblk = 0;
    double *p = nullptr, *r = nullptr, *t = nullptr, *u_best = nullptr;
    double *P1 = nullptr, *P2 = nullptr, *P3 = nullptr;
    CgState *st = nullptr;
    CgConst *cst = nullptr;
    CgMailB *mb = nullptr;
    CgMailC *mc = nullptr;
    CgState *h_st = nullptr;   // pinned
    CgConst *h_cst = nullptr;  // pinned
    // GMRES
    double *gp = nullptr, *gw = nullptr, *gx_best = nullptr, *hcol = nullptr, *rs_dev = nullptr;
    double *h_buf = nullptr;   // pinned, >= 64 doubles
};

// ---------------------------------------------------------------------------------------------
// reductions over partial arrays, identical in every workgroup
__device__ __forceinline__ double reduce_all(const double *__restrict__ part, int count, int stride, int off,
                                             double *red, bool is_max)
{
    double v = 0.0;
    for (int i = threadIdx.x; i < count; i += blockDim.x) {
        const double e = part[(size_t)i * stride + off];
        v = is_max ? fmax(v, e) : v + e;
    }
    double t = is_max ? block_max(v, red) : block_sum(v, red);
    __shared__ double bcast;
    if (threadIdx.x == 0) bcast = t;
    __syncthreads();
    t = bcast;
    __syncthreads();
    return t;
}

// r = b - A*u on rows < cap (rows >= cap: r = b), sum of squares per block -> part
__global__ __launch_bounds__(kBlock) void k_resid(const int *blk, const int *rp, const int *ci, const double *v,
                                                  const double *__restrict__ u, const double *__restrict__ b,
                                                  double *__restrict__ r, int cap, double *__restrict__ part,
                                                  const CgState *st, int gate)
{
    __shared__ SpmvSmem sm;
    if (gate && (st->skip_restore || st->iter == st->iter_best)) return;
    const double sq = csr_block_rows(blk, rp, ci, v, u, sm, [&](int row, double s) -> double {
        const double o = (cap > 0 && row >= cap) ? b[row] : b[row] + s * -1.0;
        r[row] = o;
        return o * o;
    });
    const double t = block_sum(sq, sm.red);
    if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ __launch_bounds__(1024) void k_cg_init(int n, int nblk, const double *__restrict__ part,
                                                  const double *__restrict__ r, double *__restrict__ p, double tol,
                                                  int maxit, CgState *st, CgConst *cst)
{
    __shared__ double red[16];
    const double rr = reduce_all(part, nblk, 1, 0, red, false);
    const double absres0 = sqrt(rr);
    const double normr0 = fmax(SMALLFLOAT, absres0);
    const double relres = absres0 / normr0;
    for (int i = threadIdx.x; i < n; i += 1024) p[i] = r[i];
    if (threadIdx.x == 0) {
        CgState s{};
        s.mode = relres < tol ? CG_STOP : CG_RUN;
        s.skip_restore = relres < tol;
        s.iter = 0;
        s.iter_best = 0;
        s.stag = 1;
        s.more_step = 1;
        s.absres = BIGFLOAT;
        s.absres0 = absres0;
        s.absres_best = BIGFLOAT;
        s.relres = relres;
        st[1] = s;     // iteration 1 reads st[1]
        cst->temp1 = rr;   // (z, r) with z = r
        cst->normr0 = normr0;
        cst->tol = tol;
        cst->maxdiff = tol * 1e-4;
        cst->maxit = maxit;
        cst->status = 0;
    }
}

// A: t += A*p (rows < cap), partial (t, p)
__global__ __launch_bounds__(kBlock) void k_cg_spmv(const int *blk, const int *rp, const int *ci, const double *v,
                                                    const double *__restrict__ p, double *__restrict__ t, int cap,
                                                    double *__restrict__ P1, const CgState *sin)
{
    __shared__ SpmvSmem sm;
    if (sin->mode != CG_RUN) return;
    const double c = csr_block_rows(blk, rp, ci, v, p, sm, [&](int row, double s) -> double {
        double tv = t[row];
        if (!(cap > 0 && row >= cap)) {
            tv = tv + s;
            t[row] = tv;
        }
        return tv * p[row];
    });
    const double sum = block_sum(c, sm.red);
    if (threadIdx.x == 0) P1[blockIdx.x] = sum;
}

// B: alpha; u += alpha p; r -= alpha t; partials of |r|^2, |u|^2, |p|^2, max|u|
__global__ __launch_bounds__(kBlock) void k_cg_update(int n, int nblk, const double *__restrict__ P1,
                                                      double *__restrict__ u, double *__restrict__ r,
                                                      const double *__restrict__ p, const double *__restrict__ t,
                                                      double *__restrict__ P2, const CgState *sin, const CgConst *cst,
                                                      CgMailB *mb)
{
    __shared__ double red[kBlock / 64];
    if (sin->mode != CG_RUN) return;
    const double temp2 = reduce_all(P1, nblk, 1, 0, red, false);
    const bool ok = fabs(temp2) > SMALLFLOAT2;
    const double alpha = ok ? cst->temp1 / temp2 : 0.0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        mb->alpha = alpha;
        mb->breakdown = ok ? 0 : 1;
    }
    if (!ok) return;
    const int i = blockIdx.x * kBlock + threadIdx.x;
    double rr = 0.0, uu = 0.0, pp = 0.0, um = 0.0;
    if (i < n) {
        const double pi = p[i];
        const double ui = u[i] + alpha * pi;
        const double ri = r[i] + -alpha * t[i];
        u[i] = ui;
        r[i] = ri;
        rr = ri * ri;
        uu = ui * ui;
        pp = pi * pi;
        um = fabs(ui);
    }
    double s0 = block_sum(rr, red);
    double s1 = block_sum(uu, red);
    double s2 = block_sum(pp, red);
    double s3 = block_max(um, red);
    if (threadIdx.x == 0) {
        P2[4 * blockIdx.x + 0] = s0;
        P2[4 * blockIdx.x + 1] = s1;
        P2[4 * blockIdx.x + 2] = s2;
        P2[4 * blockIdx.x + 3] = s3;
    }
}

// C: checks; best-so-far copy; residual re-computation when a convergence check fires
__global__ __launch_bounds__(kBlock) void k_cg_check(int nbe, const int *blk, const int *rp, const int *ci,
                                                     const double *v, const double *__restrict__ u,
                                                     const double *__restrict__ b, double *__restrict__ r,
                                                     double *__restrict__ u_best, int cap, const double *__restrict__ P2,
                                                     double *__restrict__ P3, const CgState *sin, const CgConst *cst,
                                                     const CgMailB *mb, CgMailC *mc)
{
    __shared__ SpmvSmem sm;
    if (sin->mode != CG_RUN || mb->breakdown) return;
    const double rr = reduce_all(P2, nbe, 4, 0, sm.red, false);
    const double uu = reduce_all(P2, nbe, 4, 1, sm.red, false);
    const double pp = reduce_all(P2, nbe, 4, 2, sm.red, false);
    const double um = reduce_all(P2, nbe, 4, 3, sm.red, true);
    const double absres = sqrt(rr);
    const double relres = absres / cst->normr0;
    const int copy_best = absres < sin->absres_best - cst->maxdiff;
    const int solstag = um <= SMALLFLOAT;
    const double normu = sqrt(uu);
    const double reldiff = fabs(mb->alpha) * sqrt(pp) / normu;
    const int stag_fire = !solstag && ((sin->stag <= max_STAG) & (reldiff < cst->maxdiff));
    const int conv_check = !solstag && (stag_fire || relres < cst->tol);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        mc->absres = absres;
        mc->relres = relres;
        mc->copy_best = copy_best;
        mc->solstag = solstag;
        mc->stag_fire = stag_fire;
        mc->conv_check = conv_check;
    }
    if (copy_best) {
        const int r0 = blk[blockIdx.x], r1 = blk[blockIdx.x + 1];
        for (int i = r0 + threadIdx.x; i < r1; i += kBlock) u_best[i] = u[i];
    }
    if (!conv_check) return;
    const double sq = csr_block_rows(blk, rp, ci, v, u, sm, [&](int row, double s) -> double {
        const double o = (cap > 0 && row >= cap) ? b[row] : b[row] + s * -1.0;
        r[row] = o;
        return o * o;
    });
    const double tsum = block_sum(sq, sm.red);
    if (threadIdx.x == 0) P3[blockIdx.x] = tsum;
}

// D: decisions of checks II/III, p = z + 1.0*p, commit the state for iteration k+1
__global__ __launch_bounds__(kBlock) void k_cg_commit(int n, int nblk, int k, const double *__restrict__ r,
                                                      double *__restrict__ p, const double *__restrict__ P3,
                                                      const CgState *sin, CgState *sout, const CgConst *cst,
                                                      const CgMailB *mb, const CgMailC *mc)
{
    __shared__ double red[kBlock / 64];
    CgState s = *sin;
    if (s.mode != CG_RUN) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *sout = s;
        return;
    }
    s.iter = k;
    bool stop = false, zero_p = false;
    if (mb->breakdown) {
        stop = true;              // goto RESTORE_BESTSOL with iter = k
    } else {
        if (mc->copy_best) {
            s.absres_best = mc->absres;
            s.iter_best = k;
        }
        s.absres = mc->absres;
        s.relres = mc->relres;
        if (mc->solstag) {
            stop = true;
            s.iter = ERROR_SOLVER_SOLSTAG;
        } else {
            double a3 = 0.0, r3 = 0.0;
            if (mc->conv_check) {
                a3 = sqrt(reduce_all(P3, nblk, 1, 0, red, false));
                r3 = a3 / cst->normr0;
            }
            if (mc->stag_fire) {
                s.absres = a3;
                s.relres = r3;
                if (r3 < cst->tol) stop = true;
                else if (s.stag >= max_STAG) {
                    stop = true;
                    s.iter = ERROR_SOLVER_STAG;
                } else {
                    zero_p = true;
                    s.stag++;
                }
            }
            if (!stop && s.relres < cst->tol) {
                s.absres = a3;
                s.relres = r3;
                if (r3 < cst->tol) stop = true;
                else if (s.more_step >= max_RESTART) {
                    stop = true;
                    s.iter = ERROR_SOLVER_TOLSMALL;
                } else {
                    zero_p = true;
                    s.more_step++;
                }
            }
            if (!stop) {
                s.absres0 = s.absres;
                const int i = blockIdx.x * kBlock + threadIdx.x;
                if (i < n) p[i] = 1.0 * r[i] + 1.0 * (zero_p ? 0.0 : p[i]);
                if (k >= cst->maxit) {
                    stop = true;       // while (iter++ < matrix) fails next: iter = matrix + 1
                    s.iter = cst->maxit + 1;
                }
            }
        }
    }
    if (stop) s.mode = CG_STOP;
    if (blockIdx.x == 0 && threadIdx.x == 0) *sout = s;
}

// restore: if absres > absres_best + maxdiff then u = u_best; publish the return status
__global__ __launch_bounds__(kBlock) void k_cg_restore(int n, int nblk, double *__restrict__ u,
                                                       const double *__restrict__ u_best, const double *__restrict__ P3,
                                                       const CgState *sfin, CgConst *cst)
{
    __shared__ double red[kBlock / 64];
    const CgState s = *sfin;
    if (blockIdx.x == 0 && threadIdx.x == 0) cst->status = s.iter > cst->maxit ? ERROR_SOLVER_matrix : s.iter;
    if (s.skip_restore || s.iter == s.iter_best) return;
    const double best = sqrt(reduce_all(P3, nblk, 1, 0, red, false));
    if (s.absres > best + cst->maxdiff) {
        const int i = blockIdx.x * kBlock + threadIdx.x;
        if (i < n) u[i] = u_best[i];
    }
}

// ---------------------------------------------------------------------------------------------
// GMRES helpers
__global__ __launch_bounds__(kBlock) void k_scal(int n, double a, double *__restrict__ x)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) x[i] *= a;
}

__global__ __launch_bounds__(kBlock) void k_copy(int n, const double *__restrict__ x, double *__restrict__ y)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) y[i] = x[i];
}

// p[i] += A*p[i-1] (rows < cap)
__global__ __launch_bounds__(kBlock) void k_acc(const int *blk, const int *rp, const int *ci, const double *v,
                                                const double *__restrict__ x, double *__restrict__ y, int cap)
{
    __shared__ SpmvSmem sm;
    (void)csr_block_rows(blk, rp, ci, v, x, sm, [&](int row, double s) -> double {
        if (!(cap > 0 && row >= cap)) y[row] = y[row] + s;
        return 0.0;
    });
}

// modified Gram-Schmidt of p[i] against p[0..i-1], then normalisation; one workgroup
__global__ __launch_bounds__(1024) void k_mgs(int n, int i, double *P, double *__restrict__ hcol)
{
    __shared__ double red[16];
    __shared__ double bcast;
    double *pi = P + (size_t)i * n;
    for (int j = 0; j < i; ++j) {
        const double *pj = P + (size_t)j * n;
        double d = 0.0;
        for (int e = threadIdx.x; e < n; e += 1024) d += pj[e] * pi[e];
        d = block_sum(d, red);
        if (threadIdx.x == 0) { bcast = d; hcol[j] = d; }
        __syncthreads();
        const double h = bcast;
        __syncthreads();
        for (int e = threadIdx.x; e < n; e += 1024) pi[e] += -h * pj[e];
        __syncthreads();
    }
    double d = 0.0;
    for (int e = threadIdx.x; e < n; e += 1024) d += pi[e] * pi[e];
    d = block_sum(d, red);
    if (threadIdx.x == 0) { bcast = sqrt(d); hcol[i] = bcast; }
    __syncthreads();
    const double t = bcast;
    if (t != 0.0) {
        const double inv = 1.0 / t;
        for (int e = threadIdx.x; e < n; e += 1024) pi[e] *= inv;
    }
}

// w = rs[i-1]*p[i-1] + sum_{j=i-2..0} rs[j]*p[j] (reference order); x += 1.0*w; optional x_best = x
__global__ __launch_bounds__(kBlock) void k_gm_update(int n, int i, const double *__restrict__ P,
                                                      const double *__restrict__ rs, double *__restrict__ x,
                                                      double *__restrict__ x_best, int copy_best)
{
    const int e = blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    double w = P[(size_t)(i - 1) * n + e];
    w *= rs[i - 1];
    for (int j = i - 2; j >= 0; --j) w += rs[j] * P[(size_t)j * n + e];
    const double xe = x[e] + 1.0 * w;
    x[e] = xe;
    if (copy_best) x_best[e] = xe;
}

// p[i] += (rs[i]-1) p[i]; p[i] += rs[j] p[j] (j = i-1..1); p[0] += (rs[0]-1) p[0]; p[0] += p[i]
__global__ __launch_bounds__(kBlock) void k_gm_recombine(int n, int i, double *__restrict__ P,
                                                         const double *__restrict__ rs)
{
    const int e = blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    double pi = P[(size_t)i * n + e];
    pi += (rs[i] - 1.0) * pi;
    for (int j = i - 1; j > 0; --j) pi += rs[j] * P[(size_t)j * n + e];
    P[(size_t)i * n + e] = pi;
    double p0 = P[e];
    p0 += (rs[0] - 1.0) * p0;
    p0 += 1.0 * pi;
    P[e] = p0;
}

// ---------------------------------------------------------------------------------------------
CoarseKrylov *coarse_krylov_create(const DevCSR &A, int row_cap, hipStream_t)
{
    auto *k = new CoarseKrylov();
    const int n = A.n;
    k->n = n;
    k->cap = row_cap;
    k->nbe = (n + kBlock - 1) / kBlock;
    k->nblk = A.nblk;
    k->p = dev_alloc<double>(n);
    k->r = dev_alloc<double>(n);
    k->t = dev_alloc<double>(n);
    k->u_best = dev_alloc<double>(n);
    k->P1 = dev_alloc<double>(A.nblk);
    k->P2 = dev_alloc<double>(4 * (size_t)k->nbe);
    k->P3 = dev_alloc<double>(A.nblk);
    k->st = dev_alloc<CgState>(2);
    k->cst = dev_alloc<CgConst>(1);
    k->mb = dev_alloc<CgMailB>(1);
    k->mc = dev_alloc<CgMailC>(1);
    k->gp = dev_alloc<double>((size_t)(max_RESTART + 1) * n);
    k->gw = dev_alloc<double>(n);
    k->gx_best = dev_alloc<double>(n);
    k->hcol = dev_alloc<double>(max_RESTART + 2);
    k->rs_dev = dev_alloc<double>(max_RESTART + 2);
    bool ok = k->p && k->r && k->t && k->u_best && k->P1 && k->P2 && k->P3 && k->st && k->cst && k->mb && k->mc &&
              k->gp && k->gw && k->gx_best && k->hcol && k->rs_dev;
    ok = ok && hipHostMalloc((void **)&k->h_st, sizeof(CgState)) == hipSuccess;
    ok = ok && hipHostMalloc((void **)&k->h_cst, sizeof(CgConst)) == hipSuccess;
    ok = ok && hipHostMalloc((void **)&k->h_buf, sizeof(double) * 64) == hipSuccess;
    if (!ok) {
        coarse_krylov_destroy(k);
        return nullptr;
    }
    return k;
}

void coarse_krylov_destroy(CoarseKrylov *k)
{
    if (!k) return;
    for (void *p : {(void *)k->p, (void *)k->r, (void *)k->t, (void *)k->u_best, (void *)k->P1, (void *)k->P2,
                    (void *)k->P3, (void *)k->st, (void *)k->cst, (void *)k->mb, (void *)k->mc, (void *)k->gp,
                    (void *)k->gw, (void *)k->gx_best, (void *)k->hcol, (void *)k->rs_dev})
        dev_free(p);
    if (k->h_st) (void)hipHostFree(k->h_st);
    if (k->h_cst) (void)hipHostFree(k->h_cst);
    if (k->h_buf) (void)hipHostFree(k->h_buf);
    delete k;
}

// sum of squares of r = b - A*u (rows < cap), read back to the host
static int host_resid_norm(CoarseKrylov *k, const DevCSR &A, const double *u, const double *b, double *r,
                           double *out, hipStream_t s)
{
    hipLaunchKernelGGL(k_resid, dim3(A.nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, u, b, r, k->cap, k->P3,
                       k->st, 0);
    int rc = launch_final_sum(k->P3, A.nblk, k->rs_dev + max_RESTART + 1, true, s);
    if (rc) return rc;
    SSS_HIP(hipMemcpyAsync(k->h_buf, k->rs_dev + max_RESTART + 1, sizeof(double), hipMemcpyDeviceToHost, s));
    SSS_HIP(hipStreamSynchronize(s));
    *out = k->h_buf[0];
    return 0;
}

static int run_cg(CoarseKrylov *k, const DevCSR &A, const double *b, double *u, double tol, int maxit, hipStream_t s,
                  int *status)
{
    const int n = k->n, nbe = k->nbe, nblk = A.nblk;
    SSS_HIP(hipMemsetAsync(k->t, 0, sizeof(double) * n, s));
    SSS_HIP(hipMemsetAsync(k->u_best, 0, sizeof(double) * n, s));
    hipLaunchKernelGGL(k_resid, dim3(nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, u, b, k->r, k->cap, k->P3,
                       k->st, 0);
    hipLaunchKernelGGL(k_cg_init, dim3(1), dim3(1024), 0, s, n, nblk, k->P3, k->r, k->p, tol, maxit, k->st, k->cst);
    int K = 0;
    for (int it = 1; it <= maxit; ++it) {
        CgState *sin = k->st + (it & 1), *sout = k->st + ((it + 1) & 1);
        hipLaunchKernelGGL(k_cg_spmv, dim3(nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, k->p, k->t, k->cap,
                           k->P1, sin);
        hipLaunchKernelGGL(k_cg_update, dim3(nbe), dim3(kBlock), 0, s, n, nblk, k->P1, u, k->r, k->p, k->t, k->P2, sin,
                           k->cst, k->mb);
        hipLaunchKernelGGL(k_cg_check, dim3(nblk), dim3(kBlock), 0, s, nbe, A.blk, A.rp, A.ci, A.v, u, b, k->r,
                           k->u_best, k->cap, k->P2, k->P3, sin, k->cst, k->mb, k->mc);
        hipLaunchKernelGGL(k_cg_commit, dim3(nbe), dim3(kBlock), 0, s, n, nblk, it, k->r, k->p, k->P3, sin, sout,
                           k->cst, k->mb, k->mc);
        K = it;
        if (it % kPoll == 0 || it == maxit || it == 1) {
            SSS_HIP(hipMemcpyAsync(k->h_st, sout, sizeof(CgState), hipMemcpyDeviceToHost, s));
            SSS_HIP(hipStreamSynchronize(s));
            if (k->h_st->mode != CG_RUN) break;
        }
    }
    CgState *sfin = k->st + ((K + 1) & 1);
    hipLaunchKernelGGL(k_resid, dim3(nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, k->u_best, b, k->r, k->cap,
                       k->P3, sfin, 1);
    hipLaunchKernelGGL(k_cg_restore, dim3(nbe), dim3(kBlock), 0, s, n, nblk, u, k->u_best, k->P3, sfin, k->cst);
    SSS_HIP(hipGetLastError());
    SSS_HIP(hipMemcpyAsync(k->h_cst, k->cst, sizeof(CgConst), hipMemcpyDeviceToHost, s));
    SSS_HIP(hipStreamSynchronize(s));
    *status = k->h_cst->status;
    return 0;
}

static int run_gmres(CoarseKrylov *k, const DevCSR &A, const double *b, double *x, double tol, int maxit,
                     hipStream_t s, int *status)
{
    const int n = k->n, restart = max_RESTART, nbe = k->nbe;
    const double maxdiff = tol * 1e-4;
    double hh[max_RESTART + 1][max_RESTART] = {}, c[max_RESTART] = {}, sn[max_RESTART] = {}, rs[max_RESTART + 1] = {};
    double r_norm, normr0, absres = BIGFLOAT, relres, absres_best = BIGFLOAT, t, gamma;
    int iter = 0, iter_best = 0, i = 0, rc;
    double *P = k->gp;
    auto pv = [&](int q) { return P + (size_t)q * n; };

    SSS_HIP(hipMemsetAsync(P, 0, sizeof(double) * (size_t)(restart + 1) * n, s));
    SSS_HIP(hipMemsetAsync(k->gx_best, 0, sizeof(double) * n, s));
    if ((rc = host_resid_norm(k, A, x, b, pv(0), &r_norm, s))) return rc;
    normr0 = fmax(SMALLFLOAT, r_norm);
    relres = r_norm / normr0;
    if (relres < tol) {
        *status = 0;
        return 0;
    }
    while (iter < maxit) {
        rs[0] = r_norm;
        hipLaunchKernelGGL(k_scal, dim3(nbe), dim3(kBlock), 0, s, n, 1.0 / r_norm, pv(0));
        i = 0;
        while (i < restart && iter < maxit) {
            i++;
            iter++;
            hipLaunchKernelGGL(k_acc, dim3(A.nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, pv(i - 1), pv(i), k->cap);
            hipLaunchKernelGGL(k_mgs, dim3(1), dim3(1024), 0, s, n, i, P, k->hcol);
            SSS_HIP(hipMemcpyAsync(k->h_buf, k->hcol, sizeof(double) * (i + 1), hipMemcpyDeviceToHost, s));
            SSS_HIP(hipStreamSynchronize(s));
            for (int j = 0; j <= i; ++j) hh[j][i - 1] = k->h_buf[j];
            for (int j = 1; j < i; ++j) {
                t = hh[j - 1][i - 1];
                hh[j - 1][i - 1] = sn[j - 1] * hh[j][i - 1] + c[j - 1] * t;
                hh[j][i - 1] = -sn[j - 1] * t + c[j - 1] * hh[j][i - 1];
            }
            t = hh[i][i - 1] * hh[i][i - 1];
            t += hh[i - 1][i - 1] * hh[i - 1][i - 1];
            gamma = sqrt(t);
            if (gamma == 0.0) gamma = SMALLFLOAT;
            c[i - 1] = hh[i - 1][i - 1] / gamma;
            sn[i - 1] = hh[i][i - 1] / gamma;
            rs[i] = -sn[i - 1] * rs[i - 1];
            rs[i - 1] = c[i - 1] * rs[i - 1];
            hh[i - 1][i - 1] = sn[i - 1] * hh[i][i - 1] + c[i - 1] * hh[i - 1][i - 1];
            absres = r_norm = fabs(rs[i]);
            relres = absres / normr0;
            if (relres <= tol) break;
        }
        rs[i - 1] = rs[i - 1] / hh[i - 1][i - 1];
        for (int q = i - 2; q >= 0; q--) {
            t = 0.0;
            for (int j = q + 1; j < i; j++) t -= hh[q][j] * rs[j];
            t += rs[q];
            rs[q] = t / hh[q][q];
        }
        const int copy_best = absres < absres_best - maxdiff;
        if (copy_best) {
            absres_best = absres;
            iter_best = iter;
        }
        std::memcpy(k->h_buf, rs, sizeof(double) * (max_RESTART + 1));
        SSS_HIP(hipMemcpyAsync(k->rs_dev, k->h_buf, sizeof(double) * (max_RESTART + 1), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_gm_update, dim3(nbe), dim3(kBlock), 0, s, n, i, P, k->rs_dev, x, k->gx_best, copy_best);
        if (relres <= tol) {
            if ((rc = host_resid_norm(k, A, x, b, k->gw, &r_norm, s))) return rc;
            absres = r_norm;
            relres = absres / normr0;
            if (relres <= tol) break;
            hipLaunchKernelGGL(k_copy, dim3(nbe), dim3(kBlock), 0, s, n, k->gw, pv(0));
            i = 0;
        }
        for (int j = i; j > 0; j--) {
            rs[j - 1] = -sn[j - 1] * rs[j];
            rs[j] = c[j - 1] * rs[j];
        }
        if (i) {
            SSS_HIP(hipStreamSynchronize(s));   // rs_dev may still be read by k_gm_update
            std::memcpy(k->h_buf, rs, sizeof(double) * (max_RESTART + 1));
            SSS_HIP(hipMemcpyAsync(k->rs_dev, k->h_buf, sizeof(double) * (max_RESTART + 1), hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_gm_recombine, dim3(nbe), dim3(kBlock), 0, s, n, i, P, k->rs_dev);
        }
    }
    if (iter != iter_best) {
        double best;
        if ((rc = host_resid_norm(k, A, k->gx_best, b, k->gw, &best, s))) return rc;
        if (absres > best + maxdiff)
            hipLaunchKernelGGL(k_copy, dim3(nbe), dim3(kBlock), 0, s, n, k->gx_best, x);
    }
    SSS_HIP(hipGetLastError());
    SSS_HIP(hipStreamSynchronize(s));
    *status = iter >= maxit ? ERROR_SOLVER_matrix : iter;
    return 0;
}

int coarse_krylov_solve(CoarseKrylov *k, const DevCSR &A, const double *b, double *x, double ctol, hipStream_t s)
{
    const int n = A.n;
    const int nn = (int)(int)((long long)n * n);
    const int maxit = std::max(250, std::min(nn, 1000));
    int status = 0, rc;
    if ((rc = run_cg(k, A, b, x, ctol, maxit, s, &status))) return rc;
    if (status < 0 && (rc = run_gmres(k, A, b, x, ctol, maxit, s, &status))) return rc;
    if (status < 0 && getenv("SSS_HIP_WARN_COARSE")) printf("### WARNING: Coarse level solver failed to converge!\n");
    return 0;
}

}  // namespace sss
