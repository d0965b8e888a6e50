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
//
// Bitwise parity.  With beta == 1 the reference CG is not a contraction: it amplifies rounding
// differences (on 1138_bus it "fails" every cycle and GMRES finishes).  Reordered reductions
// would therefore not be parity-grade, so every dot product / norm here is summed in the
// reference's sequential order: the products are formed in parallel (identically rounded) and
// staged in LDS, then one lane adds them in index order.  Coarse vectors are a few thousand
// entries, so a sequential sum costs ~10-20 us; the SpMVs are the row-exact CSR-adaptive
// kernels.  Result: the coarse solution is bitwise identical to the host reference.
//
// Control flow: CG runs device-side — per iteration one multi-workgroup SpMV (t += A*p), one
// single-workgroup step kernel (alpha, updates, norms, checks; it owns the scalar state), and a
// gated residual re-computation pair that only does work when a convergence check fires.  The
// host polls the stop flag every 32 iterations.  GMRES is host-steered: the Hessenberg column
// of each Arnoldi step is read back (i+1 doubles) and the Givens recurrences run on the host in
// the reference's exact arithmetic.
#include "sss_engine.hpp"
#include "sss_spmv_dev.hpp"

#include <cmath>
#include <cstring>
#include <vector>

namespace sss {

enum { CG_RUN = 0, CG_STOP = 1 };
constexpr int kPoll = 32;
constexpr int kSeqBlock = 1024;       // single-workgroup kernels
constexpr int kSeqChunk = 4096;       // doubles per sequential-sum LDS region (32 KiB)

struct CgState {
    int mode, iter, iter_best, stag, more_step, skip_restore, flag_resid, stag_fire, status, maxit;
    double temp1, normr0, tol, maxdiff, alpha, absres, absres0, absres_best, relres;
};

struct CoarseKrylov {
    int n = 0, cap = 0;
    double *p = nullptr, *r = nullptr, *t = nullptr, *u_best = nullptr;
    CgState *st = nullptr;
    CgState *h_st = nullptr;   // pinned
    double *gp = nullptr, *gw = nullptr, *gx_best = nullptr, *hcol = nullptr, *rs_dev = nullptr, *scal = nullptr;
    double *h_buf = nullptr;   // pinned, >= 64 doubles
};

// ---------------------------------------------------------------------------------------------
// Sequential-order sums inside one workgroup.  Up to three independent sums run concurrently
// (lanes 0, 64, 128 — three waves); each region holds one chunk of products.
struct SeqSmem {
    alignas(16) double reg[3][kSeqChunk];
    double bcast[4];
};

// s + buf[0] + buf[1] + ... in order; the pipelined chain hides the LDS read latency (the
// additions and their order are unchanged; k_cg_step at 400^3 77.6 -> 72.0 us, k_mgs 469 -> 367)
__device__ __forceinline__ double seq_add_chunk(double s, const double *buf, int m)
{
    return chain_pipe16<false>(s, buf, 0, m);
}

// returns sum_i x_i*y_i in index order (valid in every thread)
template <int NS>
__device__ void seq_dots(int n, const double *const (&xs)[NS], const double *const (&ys)[NS], double (&out)[NS],
                         SeqSmem &sm)
{
    double s = 0.0;    // lane q*64 owns sum q
    for (int base = 0; base < n; base += kSeqChunk) {
        const int m = min(kSeqChunk, n - base);
        for (int q = 0; q < NS; ++q)
            for (int i = threadIdx.x; i < m; i += blockDim.x) sm.reg[q][i] = xs[q][base + i] * ys[q][base + i];
        __syncthreads();
        for (int q = 0; q < NS; ++q)
            if ((int)threadIdx.x == q * 64) s = seq_add_chunk(s, sm.reg[q], m);
        __syncthreads();
    }
    for (int q = 0; q < NS; ++q)
        if ((int)threadIdx.x == q * 64) sm.bcast[q] = s;
    __syncthreads();
    for (int q = 0; q < NS; ++q) out[q] = sm.bcast[q];
    __syncthreads();
}

__device__ double seq_dot1(int n, const double *x, const double *y, SeqSmem &sm)
{
    const double *xs[1] = {x}, *ys[1] = {y};
    double o[1];
    seq_dots<1>(n, xs, ys, o, sm);
    return o[0];
}

__device__ double block_absmax(int n, const double *x, SeqSmem &sm)
{
    double m = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) m = fmax(m, fabs(x[i]));
    for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sm.reg[0][threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t = fmax(t, sm.reg[0][w]);
        sm.bcast[3] = t;
    }
    __syncthreads();
    const double t = sm.bcast[3];
    __syncthreads();
    return t;
}

// ---------------------------------------------------------------------------------------------
// r = b - A*u on rows < cap (rows >= cap: r = b).  gate: 0 always; 1 CG check residual (runs
// only when the step kernel asked for it); 2 CG restore (only when the best-so-far differs).
__global__ __launch_bounds__(kBlock) void k_resid(const int *blk, const int *rp, const int *ci, const double *v,
                                                  const double *__restrict__ u, const double *__restrict__ b,
                                                  double *__restrict__ r, int cap, const CgState *st, int gate)
{
    __shared__ SpmvSmem sm;
    if (gate == 1 && (st->mode != CG_RUN || !st->flag_resid)) return;
    if (gate == 2 && (st->skip_restore || st->iter == st->iter_best)) return;
    (void)csr_block_rows(blk, rp, ci, v, u, sm, [&](int row, double s) -> double {
        r[row] = (cap > 0 && row >= cap) ? b[row] : b[row] + s * -1.0;
        return 0.0;
    });
}

// t += A*p (rows < cap)
__global__ __launch_bounds__(kBlock) void k_acc(const int *blk, const int *rp, const int *ci, const double *v,
                                                const double *__restrict__ x, double *__restrict__ y, int cap,
                                                const CgState *st)
{
    __shared__ SpmvSmem sm;
    if (st && st->mode != CG_RUN) return;
    (void)csr_block_rows(blk, rp, ci, v, x, sm, [&](int row, double s) -> double {
        if (!(cap > 0 && row >= cap)) y[row] = y[row] + s;
        return 0.0;
    });
}

__global__ __launch_bounds__(kSeqBlock) void k_cg_init(int n, const double *__restrict__ r, double *__restrict__ p,
                                                       double tol, int maxit, CgState *st)
{
    __shared__ SeqSmem sm;
    const double rr = seq_dot1(n, r, r, sm);
    const double absres0 = sqrt(rr);
    const double normr0 = fmax(SMALLFLOAT, absres0);
    const double relres = absres0 / normr0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = r[i];
    if (threadIdx.x == 0) {
        CgState s;
        memset(&s, 0, sizeof(s));
        s.mode = relres < tol ? CG_STOP : CG_RUN;
        s.skip_restore = relres < tol;
        s.stag = 1;
        s.more_step = 1;
        s.maxit = maxit;
        s.temp1 = rr;          // (z, r) with z = r; frozen (as compiled)
        s.normr0 = normr0;
        s.tol = tol;
        s.maxdiff = tol * 1e-4;
        s.absres = BIGFLOAT;
        s.absres0 = absres0;
        s.absres_best = BIGFLOAT;
        s.relres = relres;
        *st = s;
    }
}

// The step's scalar part (thread 0): iteration counters, best-so-far, check I and the II/III
// triggers.  flags[0]: copy u to u_best; flags[1]: p = z + p now (no residual check pending);
// flags[2]: a residual check is pending (k_resid gate 1 + k_cg_fix).
__device__ void cg_step_state(CgState *st, int k, double alpha, const double (&sq)[3], double infnormu, int *flags)
{
    CgState s = *st;
    s.iter = k;
    s.alpha = alpha;
    s.absres = sqrt(sq[0]);
    s.relres = s.absres / s.normr0;
    int copy_best = 0;
    if (s.absres < s.absres_best - s.maxdiff) {
        s.absres_best = s.absres;
        s.iter_best = k;
        copy_best = 1;
    }
    s.flag_resid = 0;
    s.stag_fire = 0;
    if (infnormu <= SMALLFLOAT) {
        s.iter = ERROR_SOLVER_SOLSTAG;
        s.mode = CG_STOP;
    } else {
        const double normu = sqrt(sq[1]);
        const double reldiff = fabs(alpha) * sqrt(sq[2]) / normu;
        s.stag_fire = (s.stag <= max_STAG) & (reldiff < s.maxdiff);
        s.flag_resid = s.stag_fire || s.relres < s.tol;
    }
    const int finish_here = s.mode == CG_RUN && !s.flag_resid;
    if (finish_here) {
        s.absres0 = s.absres;
        if (k >= s.maxit) {               // while (iter++ < matrix) ends: iter = matrix + 1
            s.mode = CG_STOP;
            s.iter = s.maxit + 1;
        }
    }
    *st = s;
    flags[0] = copy_best;
    flags[1] = finish_here;
    flags[2] = s.mode == CG_RUN && s.flag_resid;
}

__device__ void cg_fix_body(int n, int k, const double *__restrict__ r, double *__restrict__ p, CgState *st,
                            SeqSmem &sm, int &s_pmode);

// The CG step after t += A*p: alpha, updates, norms, best-so-far, checks I and II/III triggers.
__global__ __launch_bounds__(kSeqBlock) void k_cg_step(int n, int k, double *__restrict__ u, double *__restrict__ r,
                                                       double *__restrict__ p, const double *__restrict__ t,
                                                       double *__restrict__ u_best, CgState *st)
{
    __shared__ SeqSmem sm;
    __shared__ int s_flags[3];
    if (st->mode != CG_RUN) return;
    const double temp2 = seq_dot1(n, t, p, sm);
    if (!(fabs(temp2) > SMALLFLOAT2)) {                 // possible breakdown: goto RESTORE_BESTSOL
        if (threadIdx.x == 0) { st->mode = CG_STOP; st->iter = k; }
        return;
    }
    const double alpha = st->temp1 / temp2;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        u[i] = u[i] + alpha * p[i];
        r[i] = r[i] + -alpha * t[i];
    }
    __syncthreads();
    const double *xs[3] = {r, u, p}, *ys[3] = {r, u, p};
    double sq[3];
    seq_dots<3>(n, xs, ys, sq, sm);
    const double infnormu = block_absmax(n, u, sm);
    if (threadIdx.x == 0) cg_step_state(st, k, alpha, sq, infnormu, s_flags);
    __syncthreads();
    if (s_flags[0])
        for (int i = threadIdx.x; i < n; i += blockDim.x) u_best[i] = u[i];
    if (s_flags[1])
        for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 1.0 * r[i] + 1.0 * p[i];
}

// k_cg_step for n <= kRegVec * kSeqBlock (the usual coarsest grid): t, p, u, r are read once into
// registers with every load in flight, the updated u / r / p are written from registers, and the
// infinity norm of u is reduced while lanes 0 / 64 / 128 run the three chains.  When the step asks
// for a residual check (rare: checks II / III), this workgroup recomputes r = b - A*u itself (one
// thread per row, stored order from 0.0, as k_resid) and runs k_cg_fix's body, so an iteration is
// two launches instead of four.  The arithmetic and every sum's order are those of k_cg_step +
// k_resid + k_cg_fix (tests/test_gpu_parity.py, SSS_HIP_CG_REG=0 / 1).
constexpr int kRegVec = 4;
__global__ __launch_bounds__(kSeqBlock) void k_cg_step_reg(int n, int k, double *__restrict__ u,
                                                           double *__restrict__ r, double *__restrict__ p,
                                                           const double *__restrict__ t,
                                                           double *__restrict__ u_best, CgState *st,
                                                           const int *__restrict__ rp, const int *__restrict__ ci,
                                                           const double *__restrict__ v,
                                                           const double *__restrict__ b, int cap)
{
    __shared__ SeqSmem sm;
    __shared__ double s_absw[kSeqBlock / 64];
    __shared__ int s_flags[3];
    __shared__ int s_pmode;
    if (st->mode != CG_RUN) return;
    const int tid = threadIdx.x, lane = tid & 63;
    double tv[kRegVec], pv[kRegVec], uv[kRegVec], rv[kRegVec];
#pragma unroll
    for (int j = 0; j < kRegVec; ++j) {
        const int i = tid + j * kSeqBlock;
        const bool in = i < n;
        tv[j] = in ? t[i] : 0.0;
        pv[j] = in ? p[i] : 0.0;
        uv[j] = in ? u[i] : 0.0;
        rv[j] = in ? r[i] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < kRegVec; ++j) {
        const int i = tid + j * kSeqBlock;
        if (i < n) sm.reg[0][i] = tv[j] * pv[j];
    }
    __syncthreads();
    if (tid == 0) sm.bcast[0] = chain_pipe16<false>(0.0, sm.reg[0], 0, n);
    __syncthreads();
    const double temp2 = sm.bcast[0];
    if (!(fabs(temp2) > SMALLFLOAT2)) {                 // possible breakdown: goto RESTORE_BESTSOL
        if (tid == 0) { st->mode = CG_STOP; st->iter = k; }
        return;
    }
    const double alpha = st->temp1 / temp2;
    double m = 0.0;
#pragma unroll
    for (int j = 0; j < kRegVec; ++j) {
        const int i = tid + j * kSeqBlock;
        if (i < n) {
            uv[j] = uv[j] + alpha * pv[j];
            rv[j] = rv[j] + -alpha * tv[j];
            u[i] = uv[j];
            r[i] = rv[j];
            sm.reg[0][i] = rv[j] * rv[j];
            sm.reg[1][i] = uv[j] * uv[j];
            sm.reg[2][i] = pv[j] * pv[j];
            m = fmax(m, fabs(uv[j]));
        }
    }
    for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off, 64));
    if (lane == 0) s_absw[tid >> 6] = m;
    __syncthreads();
    if (tid < 192 && lane == 0) {
        sm.bcast[tid >> 6] = chain_pipe16<false>(0.0, sm.reg[tid >> 6], 0, n);
    } else if (tid == 192) {
        double a = 0.0;
        for (int w = 0; w < kSeqBlock / 64; ++w) a = fmax(a, s_absw[w]);
        sm.bcast[3] = a;
    }
    __syncthreads();
    if (tid == 0) {
        const double sq[3] = {sm.bcast[0], sm.bcast[1], sm.bcast[2]};
        cg_step_state(st, k, alpha, sq, sm.bcast[3], s_flags);
    }
    __syncthreads();
    const int copy_best = s_flags[0], finish_here = s_flags[1];
#pragma unroll
    for (int j = 0; j < kRegVec; ++j) {
        const int i = tid + j * kSeqBlock;
        if (i < n) {
            if (copy_best) u_best[i] = uv[j];
            if (finish_here) p[i] = 1.0 * rv[j] + 1.0 * pv[j];
        }
    }
    if (!s_flags[2]) return;
    // k_resid gate 1: r = b - A*u on rows < cap (u as written above; the barriers since order it)
    for (int row = tid; row < n; row += kSeqBlock) {
        if (cap > 0 && row >= cap) {
            r[row] = b[row];
            continue;
        }
        const int e = rp[row + 1];
        double acc = 0.0;
        int kk = rp[row];
        for (; kk + 4 <= e; kk += 4) {
            int c[4];
            double a[4], xv[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) c[h] = ci[kk + h], a[h] = v[kk + h];
#pragma unroll
            for (int h = 0; h < 4; ++h) xv[h] = c[h] >= 0 ? u[c[h]] : 0.0;
#pragma unroll
            for (int h = 0; h < 4; ++h) acc += c[h] >= 0 ? a[h] * xv[h] : 0.0;
        }
        for (; kk < e; ++kk) acc += ci[kk] >= 0 ? v[kk] * u[ci[kk]] : 0.0;
        r[row] = b[row] + acc * -1.0;
    }
    __syncthreads();
    cg_fix_body(n, k, r, p, st, sm, s_pmode);
}

// After the gated residual re-computation: checks II (stagnation) and III (false convergence).
// Every thread of the workgroup calls it; s_pmode is a __shared__ int.
__device__ void cg_fix_body(int n, int k, const double *__restrict__ r, double *__restrict__ p, CgState *st,
                            SeqSmem &sm, int &s_pmode)
{
    const double a3 = sqrt(seq_dot1(n, r, r, sm));
    if (threadIdx.x == 0) {
        CgState s = *st;
        bool stop = false, zero_p = false;
        const double r3 = a3 / s.normr0;
        if (s.stag_fire) {
            s.absres = a3;
            s.relres = r3;
            if (r3 < s.tol) stop = true;
            else if (s.stag >= max_STAG) { stop = true; s.iter = ERROR_SOLVER_STAG; }
            else { zero_p = true; s.stag++; }
        }
        if (!stop && s.relres < s.tol) {
            s.absres = a3;
            s.relres = r3;
            if (r3 < s.tol) stop = true;
            else if (s.more_step >= max_RESTART) { stop = true; s.iter = ERROR_SOLVER_TOLSMALL; }
            else { zero_p = true; s.more_step++; }
        }
        s_pmode = 0;
        if (!stop) {
            s.absres0 = s.absres;
            s_pmode = zero_p ? 2 : 1;
            if (k >= s.maxit) { stop = true; s.iter = s.maxit + 1; }
        }
        if (stop) s.mode = CG_STOP;
        s.flag_resid = 0;
        *st = s;
    }
    __syncthreads();
    if (s_pmode)
        for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 1.0 * r[i] + 1.0 * (s_pmode == 2 ? 0.0 : p[i]);
}

__global__ __launch_bounds__(kSeqBlock) void k_cg_fix(int n, int k, const double *__restrict__ r,
                                                      double *__restrict__ p, CgState *st)
{
    __shared__ SeqSmem sm;
    __shared__ int s_pmode;   // 0: no p update, 1: p = z + p, 2: p = z + 0
    if (st->mode != CG_RUN || !st->flag_resid) return;
    cg_fix_body(n, k, r, p, st, sm, s_pmode);
}

__global__ __launch_bounds__(kSeqBlock) void k_cg_restore(int n, double *__restrict__ u,
                                                          const double *__restrict__ u_best,
                                                          const double *__restrict__ r, CgState *st)
{
    __shared__ SeqSmem sm;
    __shared__ int s_copy;
    const CgState s0 = *st;
    if (threadIdx.x == 0) st->status = s0.iter > s0.maxit ? ERROR_SOLVER_matrix : s0.iter;
    if (s0.skip_restore || s0.iter == s0.iter_best) return;
    const double best = sqrt(seq_dot1(n, r, r, sm));
    if (threadIdx.x == 0) s_copy = s0.absres > best + s0.maxdiff;
    __syncthreads();
    if (s_copy)
        for (int i = threadIdx.x; i < n; i += blockDim.x) u[i] = u_best[i];
}

// ---------------------------------------------------------------------------------------------
// GMRES kernels (single workgroup unless noted)
__global__ __launch_bounds__(kSeqBlock) void k_seq_norm(int n, const double *__restrict__ x, double *out)
{
    __shared__ SeqSmem sm;
    const double s = sqrt(seq_dot1(n, x, x, sm));
    if (threadIdx.x == 0) *out = s;
}

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

// modified Gram-Schmidt of p[i] against p[0..i-1], then normalisation
__global__ __launch_bounds__(kSeqBlock) void k_mgs(int n, int i, double *P, double *__restrict__ hcol)
{
    __shared__ SeqSmem sm;
    double *pi = P + (size_t)i * n;
    for (int j = 0; j < i; ++j) {
        const double *pj = P + (size_t)j * n;
        const double h = seq_dot1(n, pj, pi, sm);
        if (threadIdx.x == 0) hcol[j] = h;
        for (int e = threadIdx.x; e < n; e += blockDim.x) pi[e] += -h * pj[e];
        __syncthreads();
    }
    const double t = sqrt(seq_dot1(n, pi, pi, sm));
    if (threadIdx.x == 0) hcol[i] = t;
    if (t != 0.0) {
        const double inv = 1.0 / t;
        for (int e = threadIdx.x; e < n; e += blockDim.x) pi[e] *= inv;
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
    k->p = dev_alloc<double>(n);
    k->r = dev_alloc<double>(n);
    k->t = dev_alloc<double>(n);
    k->u_best = dev_alloc<double>(n);
    k->st = dev_alloc<CgState>(1);
    k->gp = dev_alloc<double>((size_t)(max_RESTART + 1) * n);
    k->gw = dev_alloc<double>(n);
    k->gx_best = dev_alloc<double>(n);
    k->hcol = dev_alloc<double>(max_RESTART + 2);
    k->rs_dev = dev_alloc<double>(max_RESTART + 2);
    k->scal = dev_alloc<double>(2);
    bool ok = k->p && k->r && k->t && k->u_best && k->st && k->gp && k->gw && k->gx_best && k->hcol && k->rs_dev &&
              k->scal;
    ok = ok && hipHostMalloc((void **)&k->h_st, sizeof(CgState)) == hipSuccess;
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
    for (void *p : {(void *)k->p, (void *)k->r, (void *)k->t, (void *)k->u_best, (void *)k->st, (void *)k->gp,
                    (void *)k->gw, (void *)k->gx_best, (void *)k->hcol, (void *)k->rs_dev, (void *)k->scal})
        dev_free(p);
    if (k->h_st) (void)hipHostFree(k->h_st);
    if (k->h_buf) (void)hipHostFree(k->h_buf);
    delete k;
}

// r = b - A*u (rows < cap) and ||r|| (sequential order) read back to the host
static int host_resid_norm(CoarseKrylov *k, const DevCSR &A, const double *u, const double *b, double *r,
                           double *out, hipStream_t s)
{
    hipLaunchKernelGGL(k_resid, dim3(A.nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, u, b, r, k->cap,
                       (const CgState *)nullptr, 0);
    hipLaunchKernelGGL(k_seq_norm, dim3(1), dim3(kSeqBlock), 0, s, k->n, r, k->scal);
    SSS_HIP(hipMemcpyAsync(k->h_buf, k->scal, sizeof(double), hipMemcpyDeviceToHost, s));
    SSS_HIP(hipStreamSynchronize(s));
    *out = k->h_buf[0];
    return 0;
}

static int run_cg(CoarseKrylov *k, const DevCSR &A, const double *b, double *u, double tol, int maxit, hipStream_t s,
                  int *status)
{
    const int n = k->n, nblk = A.nblk;
    const char *cr = getenv("SSS_HIP_CG_REG");   // "0": the LDS-chunked step at every size (test hook)
    const bool reg_step = !(cr && cr[0] == '0') && n <= kRegVec * kSeqBlock;
    SSS_HIP(hipMemsetAsync(k->t, 0, sizeof(double) * n, s));
    SSS_HIP(hipMemsetAsync(k->u_best, 0, sizeof(double) * n, s));
    hipLaunchKernelGGL(k_resid, dim3(nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, u, b, k->r, k->cap,
                       (const CgState *)nullptr, 0);
    hipLaunchKernelGGL(k_cg_init, dim3(1), dim3(kSeqBlock), 0, s, n, k->r, k->p, tol, maxit, k->st);
    for (int it = 1; it <= maxit; ++it) {
        hipLaunchKernelGGL(k_acc, dim3(nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, k->p, k->t, k->cap,
                           (const CgState *)k->st);
        if (reg_step) {
            hipLaunchKernelGGL(k_cg_step_reg, dim3(1), dim3(kSeqBlock), 0, s, n, it, u, k->r, k->p, k->t, k->u_best,
                               k->st, A.rp, A.ci, A.v, b, k->cap);
        } else {
            hipLaunchKernelGGL(k_cg_step, dim3(1), dim3(kSeqBlock), 0, s, n, it, u, k->r, k->p, k->t, k->u_best,
                               k->st);
            hipLaunchKernelGGL(k_resid, dim3(nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, u, b, k->r, k->cap,
                               (const CgState *)k->st, 1);
            hipLaunchKernelGGL(k_cg_fix, dim3(1), dim3(kSeqBlock), 0, s, n, it, k->r, k->p, k->st);
        }
        if (it % kPoll == 0 || it == maxit || it == 1) {
            SSS_HIP(hipMemcpyAsync(k->h_st, k->st, sizeof(CgState), hipMemcpyDeviceToHost, s));
            SSS_HIP(hipStreamSynchronize(s));
            if (k->h_st->mode != CG_RUN) break;
        }
    }
    hipLaunchKernelGGL(k_resid, dim3(nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, k->u_best, b, k->r, k->cap,
                       (const CgState *)k->st, 2);
    hipLaunchKernelGGL(k_cg_restore, dim3(1), dim3(kSeqBlock), 0, s, n, u, k->u_best, k->r, k->st);
    SSS_HIP(hipGetLastError());
    SSS_HIP(hipMemcpyAsync(k->h_st, k->st, sizeof(CgState), hipMemcpyDeviceToHost, s));
    SSS_HIP(hipStreamSynchronize(s));
    *status = k->h_st->status;
    return 0;
}

static int run_gmres(CoarseKrylov *k, const DevCSR &A, const double *b, double *x, double tol, int maxit,
                     hipStream_t s, int *status)
{
    const int n = k->n, restart = max_RESTART, nbe = (n + kBlock - 1) / kBlock;
    const double maxdiff = tol * 1e-4;
    double hh[max_RESTART + 1][max_RESTART] = {}, c[max_RESTART] = {}, sn[max_RESTART] = {}, rs[max_RESTART + 1] = {};
    double r_norm, normr0, absres = BIGFLOAT, relres, absres_best = BIGFLOAT, t, gamma;
    int iter = 0, iter_best = 0, i = 0, rc;
    double *P = k->gp;
    auto pv = [&](int q) { return P + (size_t)q * n; };
    auto upload_rs = [&]() -> int {
        SSS_HIP(hipStreamSynchronize(s));   // h_buf and rs_dev may still be in use
        std::memcpy(k->h_buf, rs, sizeof(double) * (max_RESTART + 1));
        SSS_HIP(hipMemcpyAsync(k->rs_dev, k->h_buf, sizeof(double) * (max_RESTART + 1), hipMemcpyHostToDevice, s));
        return 0;
    };

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
        t = 1.0 / r_norm;
        hipLaunchKernelGGL(k_scal, dim3(nbe), dim3(kBlock), 0, s, n, t, pv(0));
        i = 0;
        while (i < restart && iter < maxit) {
            i++;
            iter++;
            hipLaunchKernelGGL(k_acc, dim3(A.nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, pv(i - 1), pv(i), k->cap,
                               (const CgState *)nullptr);
            hipLaunchKernelGGL(k_mgs, dim3(1), dim3(kSeqBlock), 0, s, n, i, P, k->hcol);
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
        if ((rc = upload_rs())) return rc;
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
            if ((rc = upload_rs())) return rc;
            hipLaunchKernelGGL(k_gm_recombine, dim3(nbe), dim3(kBlock), 0, s, n, i, P, k->rs_dev);
        }
    }
    if (iter != iter_best) {
        double best;
        if ((rc = host_resid_norm(k, A, k->gx_best, b, k->gw, &best, s))) return rc;
        if (absres > best + maxdiff) hipLaunchKernelGGL(k_copy, dim3(nbe), dim3(kBlock), 0, s, n, k->gx_best, x);
    }
    SSS_HIP(hipGetLastError());
    SSS_HIP(hipStreamSynchronize(s));
    *status = iter >= maxit ? ERROR_SOLVER_matrix : iter;
    return 0;
}

int coarse_krylov_solve(CoarseKrylov *k, const DevCSR &A, const double *b, double *x, double ctol, hipStream_t s)
{
    const int n = A.n;
    const int nn = (int)(long long)((long long)n * n);   // n*n in int, as the reference
    const int maxit = std::max(250, std::min(nn, 1000));
    int status = 0, rc;
    if ((rc = run_cg(k, A, b, x, ctol, maxit, s, &status))) return rc;
    if (status < 0 && (rc = run_gmres(k, A, b, x, ctol, maxit, s, &status))) return rc;
    if (status < 0 && getenv("SSS_HIP_WARN_COARSE")) printf("### WARNING: Coarse level solver failed to converge!\n");
    return 0;
}

}  // namespace sss
