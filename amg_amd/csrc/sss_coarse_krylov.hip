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
#include <cstdio>
#include <algorithm>
#include <queue>
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
    // the one-launch CG (k_cg_persist): {tag, half} granules of p (2 n) and t (2 n), the command
    // word and the stall word (pctl), the launch counter that makes every launch's tags fresh
    unsigned long long *gp_p = nullptr, *gp_t = nullptr, *pctl = nullptr;
    unsigned epoch = 0;
    int persist_grid = -1;  // workgroups of the one-launch CG; -1: it does not fit (two kernels per iteration)
    int *wl_ptr = nullptr, *wl_rows = nullptr;   // each worker wave's rows (cg_persist_plan)
    double *tw = nullptr;                        // t_{k-1}, t_k by parity of k (the worker's own rows)
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
// The whole CG loop in one launch (k_cg_persist; n <= kRegVec * kSeqBlock).  Workgroup 0 runs every
// step as k_cg_step_reg does (same arithmetic, same sequential sums); workgroups 1 .. G-1 run the
// SpMVs t_k = t_{k-1} + A p_k, one wave per row at a time, each row summed from 0.0 in stored order
// and added to t_{k-1} as k_acc does.  A row's sum is one dependent chain of adds issued by one lane,
// so what bounds the SpMV is the chain work each SIMD issues: the host deals the rows to the waves
// longest first onto the least-loaded SIMD (cg_persist_plan; the coarsest level of 7-pt 400^3 has
// rows of 2 to 2,907 entries, 767 on average), and each wave works through its list.  The two sides
// hand over through {tag, half} granules (8-byte agent-scope atomics, the 8 XCD L2s are not
// coherent): p_k from workgroup 0 (all rows; two buffers by command parity), t_k from the wave that
// owns the row; workgroup 0's waves 4-15 collect t chunk by chunk and wave 3 sums t.p over each run
// of ready chunks as it arrives.  A command (tag, k, exit) in a ring of four words
// starts each SpMV: a word is rewritten only after every worker has answered the command two back.
//   Speculation: with beta == 1, p_{k+1} = 1.0 r + 1.0 p_k is known as soon as alpha has updated r --
// before the step's three norm chains decide whether a residual check (rare) rewrites it.  Workgroup
// 0 publishes it right away, so SpMV k+1 overlaps the rest of step k; when the check fires, the fixed
// p_{k+1} goes out under a new tag and the workers redo SpMV k+1 from t_k: t_k lives in tw[k & 1],
// written and read only by the lane that owns the row.
//   Progress: every workgroup is co-resident (the grid is capped by the occupancy API) and every wait
// is bounded (spin polls; past the limit the stall word is set and every workgroup leaves).
#define CGP_RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
constexpr int kCgpWaves = kSeqBlock / 64;
constexpr int kCgpSpin = 1 << 20;    // polls before a waiting wave gives up (~1 s with the back-off);
                                     // SSS_HIP_CG_SPIN: another limit (test hook; negative: every wait fails)
constexpr int kCgpTraceIts = 256, kCgpTraceK = 10;
constexpr int kCgpSimds = 4;         // SIMDs per CU: a worker's 16 waves, four on each

__device__ __forceinline__ void cgp_put(unsigned long long *g, unsigned tag, double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    __hip_atomic_store(g, ((unsigned long long)tag << 32) | (u & 0xffffffffull), CGP_RLX);
    __hip_atomic_store(g + 1, ((unsigned long long)tag << 32) | (u >> 32), CGP_RLX);
}
// s + p[0] + ... + p[m-1] in order (chain_pipe16's additions, 8 products read ahead instead of 16: the
// step workgroup of k_cg_persist keeps its vectors in registers around its chains)
__device__ __forceinline__ double chain_pipe8(double s, const double *p, int m)
{
    int k = 0;
    if (m >= 16) {
        double2 c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = *reinterpret_cast<const double2 *>(p + 2 * u);
        for (k = 8; k + 8 <= m; k += 8) {
            double2 nx[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) nx[u] = *reinterpret_cast<const double2 *>(p + k + 2 * u);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                s += c[u].x;
                s += c[u].y;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = nx[u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            s += c[u].x;
            s += c[u].y;
        }
    }
    for (; k < m; ++k) s += p[k];
    return s;
}

// Granules i0 + j * stride (j < N, those below n) of base, all loads in flight before any check;
// out[j] = 0.0 past n
template <int N>
__device__ __forceinline__ void cgp_wait_n(const unsigned long long *base, int i0, int stride, int n, unsigned tag,
                                           int spin, unsigned long long *err, double (&out)[N])
{
    bool done[N];
#pragma unroll
    for (int j = 0; j < N; ++j) done[j] = i0 + j * stride >= n, out[j] = 0.0;
    for (int s = 0;; ++s) {
        unsigned long long a[N], c[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            unsigned long long *g = const_cast<unsigned long long *>(base) + 2 * (size_t)(i0 + j * stride);
            a[j] = done[j] ? 0ull : __hip_atomic_load(g, CGP_RLX);
            c[j] = done[j] ? 0ull : __hip_atomic_load(g + 1, CGP_RLX);
        }
        bool all = true;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if (done[j]) continue;
            if ((unsigned)(a[j] >> 32) == tag && (unsigned)(c[j] >> 32) == tag) {
                out[j] = __longlong_as_double((long long)((c[j] << 32) | (a[j] & 0xffffffffull)));
                done[j] = true;
            } else {
                all = false;
            }
        }
        if (all && spin >= 0) return;
        if (s >= spin || ((s & 63) == 63 && __hip_atomic_load(err, CGP_RLX))) {
            __hip_atomic_store(err, 1ull, CGP_RLX);
            return;
        }
        if (s < 32) __builtin_amdgcn_s_sleep(1);
        else __builtin_amdgcn_s_sleep(4);
    }
}
__device__ __forceinline__ unsigned cgp_tag(unsigned epoch, int seq) { return (epoch << 12) | (unsigned)seq; }

// k_cg_persist's rare residual check (k_resid gate 1 + k_cg_fix): r = b - A u on rows < cap, one
// thread per row as k_cg_step_reg; u and p_k in global memory; ends with every thread past a barrier.
__device__ __forceinline__ void cgp_check(int n, int k, const int *__restrict__ rp, const int *__restrict__ ci,
                                       const double *__restrict__ v, const double *__restrict__ b, int cap,
                                       const double *u, double *r, double *p, CgState *ss, SeqSmem &sm, int &s_pmode)
{
    for (int row = threadIdx.x; row < n; row += kSeqBlock) {
        if (cap > 0 && row >= cap) {
            r[row] = b[row];
            continue;
        }
        const int e = rp[row + 1];
        double acc = 0.0;
        int kk = rp[row];
        for (; kk + 4 <= e; kk += 4) {
            int cc[4];
            double a[4], xv[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) cc[h] = ci[kk + h], a[h] = v[kk + h];
#pragma unroll
            for (int h = 0; h < 4; ++h) xv[h] = cc[h] >= 0 ? u[cc[h]] : 0.0;
#pragma unroll
            for (int h = 0; h < 4; ++h) acc += cc[h] >= 0 ? a[h] * xv[h] : 0.0;
        }
        for (; kk < e; ++kk) acc += ci[kk] >= 0 ? v[kk] * u[ci[kk]] : 0.0;
        r[row] = b[row] + acc * -1.0;
    }
    __syncthreads();
    cg_fix_body(n, k, r, p, ss, sm, s_pmode);
    __syncthreads();
}

// 0.0 + a_k p_{c_k} over the row's entries [k0, k1) in stored order, by one wave (valid in lane 0):
// wave_row_chain's additions, with the next strip's column / value loads in flight while lane 0 chains
// the current one (two strips per wave) -- on the coarsest level of 7-pt 400^3 a row of 2,907 entries
// is the SpMV's critical path.  x from LDS (the workers' copy of p).
__device__ __forceinline__ double cgp_row_chain(int k0, int k1, const int *__restrict__ ci, const double *__restrict__ v,
                                                const double *x, double *strip0, double *strip1,
                                                unsigned long long *tacc = nullptr)
{
    constexpr int U = kWaveStage / 64;
    const int lane = threadIdx.x & 63;
    double acc = 0.0;
    if (k1 <= k0) return acc;
    int c[U];
    double a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {   // strip 0 (clamped: a lane past the row loads its last entry, value 0.0)
        const int q = lane + 64 * u, kc = min(k0 + q, k1 - 1);
        c[u] = ci[kc];
        a[u] = k0 + q < k1 ? v[kc] : 0.0;
    }
    int cur = 0;
    unsigned long long tw_load = 0, tw_chain = 0;
    for (int base = k0; base < k1; base += kWaveStage) {
        const int m = min(kWaveStage, k1 - base);
        double *buf = cur ? strip1 : strip0;
        const unsigned long long ta = tacc ? wall_clock64() : 0;
        {   // branch-free: past the row a = 0.0 and the column is clamped (those slots are never summed)
            double xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) xv[u] = x[c[u]];
#pragma unroll
            for (int u = 0; u < U; ++u) buf[lane + 64 * u] = a[u] * xv[u];
        }
        wave_sync();
        const unsigned long long tb = tacc ? wall_clock64() : 0;
        const int nb = base + kWaveStage;
        if (nb < k1) {   // the next strip's loads, in flight during the chain below
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = lane + 64 * u, kc = min(nb + q, k1 - 1);
                c[u] = ci[kc];
                a[u] = nb + q < k1 ? v[kc] : 0.0;
            }
        }
        if (lane == 0) acc = chain_fixed<false, 16>(acc, buf, m);
        if (tacc) {
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
            const unsigned long long tc = wall_clock64();
            tw_load += tb - ta, tw_chain += tc - tb;
        }
        cur ^= 1;
    }
    if (tacc && lane == 0) tacc[0] = tw_load, tacc[1] = tw_chain;
    return acc;
}

__global__ __launch_bounds__(kSeqBlock) void k_cg_persist(int n, int maxit, const int *__restrict__ rp,
                                                          const int *__restrict__ ci, const double *__restrict__ v,
                                                          const double *__restrict__ b, int cap, double *u, double *r,
                                                          double *p, double *__restrict__ u_best, CgState *st,
                                                          unsigned long long *gpp, unsigned long long *gpt,
                                                          unsigned long long *ctl, unsigned epoch,
                                                          const int *__restrict__ wl_ptr, const int *__restrict__ wl_rows,
                                                          double *tw, int spin, unsigned long long *trc)
{
    // diagnostics (SSS_HIP_CG_TRACE): 100 MHz timestamps, plain stores -- workgroup 0's phases of
    // iterations k < kCgpTraceIts (trc[16 k + j]), and for SpMV kCgpTraceK each worker's command / p
    // (trc_w[4 b + j]) and each row's start, end, strip-load and chain time (trc_r[4 row + j])
    unsigned long long *trc_w = trc ? trc + 16 * kCgpTraceIts : nullptr, *trc_r = trc ? trc_w + 4 * gridDim.x : nullptr;
    auto ts0 = [&](int k, int j) {
        if (trc && k < kCgpTraceIts) trc[16 * k + j] = wall_clock64();
    };
    __shared__ __attribute__((aligned(16))) double lds[3 * kSeqChunk + 32];   // (+ chain_fixed's over-read)
    __shared__ double s_absw[kCgpWaves];
    __shared__ int s_simd[kCgpWaves];
    __shared__ int s_flags[3];
    __shared__ int s_pmode;
    __shared__ unsigned long long s_cmd;
    __shared__ CgState ss;
    // command ring: slot (seq & 3), one 128-byte line each; then the stall word
    auto cmd_of = [&](int sq) { return ctl + 16 * (sq & 3); };
    unsigned long long *err = ctl + 64;
    const size_t pbuf = 2 * (size_t)n;   // p granules of commands of parity 1 at gpp + pbuf
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (blockIdx.x > 0) {   // ---- a worker: SpMVs of the rows the plan gives each wave
        // p in LDS (n <= kSeqChunk), then two strips of kWaveStage per wave
        double *pl = lds, *strip0 = lds + kSeqChunk + wave * 2 * kWaveStage, *strip1 = strip0 + kWaveStage;
        // this wave's plan slot: 4 s + (its rank among the waves on SIMD s), by HW_ID [5:4]; the
        // wave index itself should the 16 waves not sit four to a SIMD
        if (lane == 0) s_simd[wave] = (__builtin_amdgcn_s_getreg(4 | (15 << 11)) >> 4) & 3;
        __syncthreads();
        int rank = 0, cnt[kCgpSimds] = {0, 0, 0, 0};
        const int mine = s_simd[wave];
        for (int w = 0; w < kCgpWaves; ++w) {
            const int sw = s_simd[w];
            rank += (w < wave && sw == mine);
            cnt[0] += sw == 0, cnt[1] += sw == 1, cnt[2] += sw == 2, cnt[3] += sw == 3;
        }
        constexpr int per = kCgpWaves / kCgpSimds;
        const bool four = cnt[0] == per && cnt[1] == per && cnt[2] == per && cnt[3] == per;
        const int gw = (int)(blockIdx.x - 1) * kCgpWaves + (four ? mine * per + rank : wave);
        const int q0 = wl_ptr[gw], q1 = wl_ptr[gw + 1];
        for (int seq = 1;; ++seq) {
            const unsigned tag = cgp_tag(epoch, seq);
            if (tid == 0) {   // the next command: tag in the high word, k << 1 | exit in the low
                unsigned long long c = 0;
                for (int s = 0;; ++s) {
                    c = __hip_atomic_load(cmd_of(seq), CGP_RLX);
                    if ((unsigned)(c >> 32) == tag && spin >= 0) break;
                    if (s >= spin || ((s & 63) == 63 && __hip_atomic_load(err, CGP_RLX))) {
                        __hip_atomic_store(err, 1ull, CGP_RLX);
                        c = ((unsigned long long)tag << 32) | 1ull;
                        break;
                    }
                    if (s < 32) __builtin_amdgcn_s_sleep(1);
                    else __builtin_amdgcn_s_sleep(4);
                }
                s_cmd = c;
            }
            __syncthreads();
            const unsigned long long c = s_cmd;
            if ((c & 1ull) || __hip_atomic_load(err, CGP_RLX)) break;
            const int k = (int)((c & 0xffffffffull) >> 1);
            const bool tr = trc && k == kCgpTraceK;
            if (tr && tid == 0) trc_w[4 * blockIdx.x] = wall_clock64();
            {
                double pw[kRegVec];
                cgp_wait_n<kRegVec>(gpp + (seq & 1) * pbuf, tid, kSeqBlock, n, tag, spin, err, pw);
#pragma unroll
                for (int q = 0; q < kRegVec; ++q)
                    if (tid + q * kSeqBlock < n) pl[tid + q * kSeqBlock] = pw[q];
            }
            __syncthreads();
            if (tr && tid == 0) trc_w[4 * blockIdx.x + 1] = wall_clock64();
            for (int q = q0; q < q1; ++q) {
                const int row = wl_rows[q];
                const bool capped = cap > 0 && row >= cap;   // t stays t_0 = 0 (k_acc's row cap)
                const unsigned long long t_row = wall_clock64();
                const double s = capped ? 0.0
                                        : cgp_row_chain(rp[row], rp[row + 1], ci, v, pl, strip0, strip1,
                                                        tr ? trc_r + 4 * row + 2 : nullptr);
                if (lane == 0) {
                    const double tprev = k > 1 ? tw[(size_t)((k - 1) & 1) * n + row] : 0.0;
                    const double tcur = capped ? tprev : tprev + s;
                    tw[(size_t)(k & 1) * n + row] = tcur;
                    cgp_put(gpt + 2 * (size_t)row, tag, tcur);
                    if (tr) {
                        trc_r[4 * row] = t_row;
                        trc_r[4 * row + 1] = wall_clock64();
                        // HW_ID: wave [3:0], SIMD [5:4], CU [11:8], SE [15:13]
                        trc_r[4 * n + row] = (unsigned)__builtin_amdgcn_s_getreg(4 | (15 << 11)) | ((unsigned long long)gw << 32);
                    }
                }
            }
        }
        return;
    }
    // ---- workgroup 0: the CG steps (k_cg_step_reg + k_resid gate 1 + k_cg_fix), p and t via granules.
    // Step k's three norm chains (waves 0-2) run while waves 4-15 collect t_{k+1} of the speculative
    // SpMV chunk by chunk in index order, each chunk as t_{k+1} p_{k+1} into LDS with a ready flag, and
    // wave 3 chains the chunks as they turn ready: the chain runs behind the SpMV's rows instead of
    // after the last of them, and the next step's (t, p) starts ready.
    SeqSmem &sm = *reinterpret_cast<SeqSmem *>(lds);
    constexpr int kTpChunk = 128, kTpChunks = kSeqChunk / kTpChunk, kTpPollers = kCgpWaves - 4;
    __shared__ __attribute__((aligned(16))) double tp[kSeqChunk + 16];   // p_{k+1}, then t_{k+1} * p_{k+1}
    __shared__ int s_rdy[kTpChunks];   // chunk c of round r summed-ready when s_rdy[c] == r
    __shared__ double s_temp2;
    const int ntp = (n + kTpChunk - 1) / kTpChunk;
    if (tid == 0) ss = *st;
    if (tid < kTpChunks) s_rdy[tid] = 0;
    __syncthreads();
    // u and r stay in global memory (each thread reads and writes its own entries: L2 hits), p_{k+1}
    // and t_k in registers -- the step's chains then run without spilling the vectors
    double tv[kRegVec], pv[kRegVec];
#pragma unroll
    for (int j = 0; j < kRegVec; ++j) {
        const int i = tid + j * kSeqBlock;
        pv[j] = i < n ? p[i] : 0.0;
    }
    int seq = 1;
    auto publish = [&](int sq, int k, const double (&pp)[kRegVec], bool exit, int ti) {
        const unsigned tag = cgp_tag(epoch, sq);
        if (!exit)
#pragma unroll
            for (int j = 0; j < kRegVec; ++j) {
                const int i = ti + j * kSeqBlock;
                if (i < n) cgp_put(gpp + (sq & 1) * pbuf + 2 * (size_t)i, tag, pp[j]);
            }
        if (tid == 0)
            __hip_atomic_store(cmd_of(sq), ((unsigned long long)tag << 32) | ((unsigned long long)k << 1) | (exit ? 1ull : 0ull),
                               CGP_RLX);
    };
    if (ss.mode != CG_RUN) {
        publish(seq, 0, pv, true, tid);
        return;
    }
    publish(seq, 1, pv, false, tid);   // SpMV 1 from p_1 (k_cg_init)
    bool spec_out = false;        // a command past `seq` is out (the speculative SpMV k + 1)
    bool have_temp2 = false;      // (t_k, p_k) already summed (behind the previous step's norms)
    double temp2 = 0.0;
    int rounds = 0;               // speculative rounds completed (chunk flags of the next one: rounds + 1)
    for (int k = 1;; ++k) {
        // the thread's index, opaque to the compiler inside the loop: the addresses of its entries
        // (u, r, p, u_best, the granules: 7 arrays x 4 entries x 64 bits) are recomputed in the
        // iteration instead of held -- and spilled -- across it
        int tid_k = tid;
        asm volatile("" : "+v"(tid_k));
        spec_out = false;   // the command at `seq` is this iteration's SpMV; none past it yet
        if (tid == 0) ts0(k, 0);
        cgp_wait_n<kRegVec>(gpt, tid_k, kSeqBlock, n, cgp_tag(epoch, seq), spin, err, tv);
        if (tid == 0) ts0(k, 1);
        if (__hip_atomic_load(err, CGP_RLX)) break;
        if (!have_temp2) {   // -- (t_k, p_k) as k_cg_step_reg sums it
#pragma unroll
            for (int j = 0; j < kRegVec; ++j) {
                const int i = tid_k + j * kSeqBlock;
                if (i < n) sm.reg[0][i] = tv[j] * pv[j];
            }
            __syncthreads();
            if (tid == 0) s_temp2 = chain_fixed<false, 8>(0.0, sm.reg[0], n);
            __syncthreads();
            temp2 = s_temp2;
        }
        have_temp2 = false;
        if (!(fabs(temp2) > SMALLFLOAT2)) {   // possible breakdown: goto RESTORE_BESTSOL
            if (tid == 0) {
                ss.mode = CG_STOP;
                ss.iter = k;
            }
            break;
        }
        const double alpha = ss.temp1 / temp2;
        double m = 0.0;
#pragma unroll
        for (int j = 0; j < kRegVec; ++j) {
            const int i = tid_k + j * kSeqBlock;
            if (i < n) {
                const double un = u[i] + alpha * pv[j];
                const double rn = r[i] + -alpha * tv[j];
                u[i] = un;
                r[i] = rn;
                m = fmax(m, fabs(un));
                sm.reg[0][i] = rn * rn;
                sm.reg[1][i] = un * un;
                sm.reg[2][i] = pv[j] * pv[j];
                p[i] = pv[j];                    // p_k, for a residual check that rewrites p_{k+1}
                pv[j] = 1.0 * rn + 1.0 * pv[j];  // p_{k+1} if none does
                tp[i] = pv[j];
            } else {
                pv[j] = 0.0;
            }
        }
        if (tid == 0) ts0(k, 2);
        spec_out = k < ss.maxit;   // (at maxit the step always stops)
        if (spec_out) publish(seq + 1, k + 1, pv, false, tid_k);
        if (tid == 0) ts0(k, 3);
        for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off, 64));
        if (lane == 0) s_absw[wave] = m;
        __syncthreads();
        if (tid < 192) {   // the norms of step k
            if (lane == 0) sm.bcast[wave] = chain_fixed<false, 8>(0.0, sm.reg[wave], n);
        } else if (tid < 256) {   // wave 3: the absmax, then t_{k+1} p_{k+1} chunk by chunk as they turn ready
            if (lane == 0) {
                double a = 0.0;
                for (int w = 0; w < kCgpWaves; ++w) a = fmax(a, s_absw[w]);
                sm.bcast[3] = a;
                if (spec_out) {
                    if (trc) ts0(k, 5);
                    double s = 0.0;
                    bool gone = false;   // past a stall every later chunk is summed without waiting
                    for (int c = 0; c < ntp;) {
                        for (int sp = 0; !gone && __hip_atomic_load(&s_rdy[c], __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_WORKGROUP) <= rounds;
                             ++sp) {
                            if (sp >= spin || ((sp & 63) == 63 && __hip_atomic_load(err, CGP_RLX))) {
                                __hip_atomic_store(err, 1ull, CGP_RLX);
                                gone = true;
                            }
                            __builtin_amdgcn_s_sleep(1);
                        }
                        // and every chunk after it that is ready already: one chain over the run
                        int ce = c + 1;
                        while (ce < ntp && (gone || __hip_atomic_load(&s_rdy[ce], __ATOMIC_RELAXED,
                                                                      __HIP_MEMORY_SCOPE_WORKGROUP) > rounds))
                            ++ce;
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                        if (c == 0 && trc) ts0(k, 6);
                        if (trc && k < kCgpTraceIts) ts0(k, 8), trc[16 * k + 9] = min(ce * kTpChunk, n) - c * kTpChunk;
                        s = chain_fixed<false, 16>(s, tp + c * kTpChunk, min(ce * kTpChunk, n) - c * kTpChunk);
                        c = ce;
                    }
                    s_temp2 = s;
                    if (trc) ts0(k, 7);
                }
            }
        } else if (spec_out) {   // waves 4-15: chunks wave - 4, + 12, ... of t_{k+1} (in the chain's order)
            for (int c = wave - 4; c < ntp; c += kTpPollers) {
                double tt[kTpChunk / 64];
                cgp_wait_n<kTpChunk / 64>(gpt, c * kTpChunk + lane, 64, n, cgp_tag(epoch, seq + 1), spin, err, tt);
#pragma unroll
                for (int q = 0; q < kTpChunk / 64; ++q) {
                    const int i = c * kTpChunk + lane + 64 * q;
                    if (i < n) tp[i] = tt[q] * tp[i];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) __hip_atomic_store(&s_rdy[c], rounds + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();
        if (spec_out) ++rounds;
        if (tid == 0) {
            const double sq[3] = {sm.bcast[0], sm.bcast[1], sm.bcast[2]};
            cg_step_state(&ss, k, alpha, sq, sm.bcast[3], s_flags);
        }
        __syncthreads();
        const int copy_best = s_flags[0], finish_here = s_flags[1], check = s_flags[2];
        if (tid == 0) ts0(k, 12);
#pragma unroll
        for (int j = 0; j < kRegVec; ++j) {
            const int i = tid_k + j * kSeqBlock;
            if (i < n && copy_best) u_best[i] = u[i];
        }
        if (finish_here) {
            if (ss.mode != CG_RUN) break;   // maxit reached (no command went out)
            temp2 = s_temp2;                // (t_{k+1}, p_{k+1}): p_{k+1} = pv, already out
            have_temp2 = true;
            seq += 1;
            continue;
        }
        if (!check) break;   // stopped by the step (a speculative command may be out)
        // -- k_resid gate 1 + k_cg_fix: r = b - A u (rows < cap), checks II / III, p rewritten from
        // p_k (in p since the update)
        __syncthreads();
        cgp_check(n, k, rp, ci, v, b, cap, u, r, p, &ss, sm, s_pmode);
        if (ss.mode != CG_RUN || !s_pmode) break;
#pragma unroll
        for (int j = 0; j < kRegVec; ++j) {
            const int i = tid_k + j * kSeqBlock;
            pv[j] = i < n ? p[i] : 0.0;
        }
        // the fixed p_{k+1} under a fresh tag: the workers redo SpMV k + 1 from t_k
        seq += spec_out ? 2 : 1;
        publish(seq, k + 1, pv, false, tid_k);
        spec_out = false;
    }
    // every worker leaves at the next command
    publish(seq + (spec_out ? 2 : 1), 0, pv, true, tid);
    __syncthreads();
    if (tid == 0) *st = ss;
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
static void cg_persist_plan(CoarseKrylov *k, const DevCSR &A);

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
    k->gp_p = dev_alloc<unsigned long long>(4 * (size_t)n);   // two buffers of {tag, half} pairs
    k->gp_t = dev_alloc<unsigned long long>(2 * (size_t)n);
    k->pctl = dev_alloc<unsigned long long>(80);
    bool ok = k->p && k->r && k->t && k->u_best && k->st && k->gp && k->gw && k->gx_best && k->hcol && k->rs_dev &&
              k->scal && k->gp_p && k->gp_t && k->pctl;
    ok = ok && hipMemset(k->gp_p, 0, sizeof(unsigned long long) * 4 * (size_t)n) == hipSuccess &&
         hipMemset(k->gp_t, 0, sizeof(unsigned long long) * 2 * (size_t)n) == hipSuccess &&
         hipMemset(k->pctl, 0, sizeof(unsigned long long) * 80) == hipSuccess;
    ok = ok && hipHostMalloc((void **)&k->h_st, sizeof(CgState)) == hipSuccess;
    ok = ok && hipHostMalloc((void **)&k->h_buf, sizeof(double) * 64) == hipSuccess;
    if (ok) cg_persist_plan(k, A);
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
                    (void *)k->gw, (void *)k->gx_best, (void *)k->hcol, (void *)k->rs_dev, (void *)k->scal,
                    (void *)k->gp_p, (void *)k->gp_t, (void *)k->pctl, (void *)k->wl_ptr, (void *)k->wl_rows,
                    (void *)k->tw})
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

// The one-launch CG's plan: one step workgroup and W workers (every workgroup co-resident: the
// occupancy API bounds W), and the rows of each worker's wave slots, slot 4 s + j being the j-th
// wave on SIMD s (k_cg_persist reads each wave's SIMD from HW_ID).  A row's SpMV is a chain of
// dependent adds issued by one lane, and the waves on one SIMD share its issue slots, so rows go
// longest first onto the SIMD with the least work (entries + a per-row overhead) and within it onto
// its least-loaded slot; each list runs in ascending row order (the rows of low index are the first
// the step workgroup's t.p chain needs).  Measured at 400^3 (SSS_HIP_CG_TRACE): four chaining waves
// per SIMD finish the SpMV sooner than one wave per SIMD working through the same rows in turn, and
// balancing per SIMD beats balancing per wave (42.6 against 55.0 us per iteration).  Sets
// persist_grid = W + 1, or -1 when the one-launch form does not fit.
static void cg_persist_plan(CoarseKrylov *k, const DevCSR &A)
{
    k->persist_grid = -1;
    const int n = A.n;
    int dev = 0, per_cu = 0;
    hipDeviceProp_t prop;
    if (n < 1 || n > kRegVec * kSeqBlock || hipGetDevice(&dev) != hipSuccess ||
        hipGetDeviceProperties(&prop, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_cg_persist, kSeqBlock, 0) != hipSuccess)
        return;
    const int resident = per_cu * prop.multiProcessorCount;   // every workgroup must be co-resident
    if (resident < 2) return;
    const int workers = std::min(resident - 1, std::max(1, (n + 3) / 4)), nwaves = workers * kCgpWaves;
    std::vector<int> rp(n + 1);
    if (hipMemcpy(rp.data(), A.rp, sizeof(int) * (n + 1), hipMemcpyDeviceToHost) != hipSuccess) return;
    constexpr long long kRowCost = 64;   // per-row overhead in entries (command, strip set-up, publish)
    auto cost = [&](int r) { return (long long)(rp[r + 1] - rp[r]) + kRowCost; };
    std::vector<int> order(n);
    for (int i = 0; i < n; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost(a) > cost(b); });
    using Bin = std::pair<long long, int>;   // (load, worker * 4 + SIMD)
    std::priority_queue<Bin, std::vector<Bin>, std::greater<Bin>> simds;
    for (int b = 0; b < workers * kCgpSimds; ++b) simds.push({0, b});
    constexpr int per = kCgpWaves / kCgpSimds;
    // chaining waves per SIMD (SSS_HIP_CG_CHAINERS, 1..4): measured against each other at 400^3
    int chainers = per;
    if (const char *e = getenv("SSS_HIP_CG_CHAINERS")) chainers = std::max(1, std::min(per, atoi(e)));
    std::vector<long long> sload(nwaves, 0);
    std::vector<std::vector<int>> lists(nwaves);
    for (int r : order) {
        Bin b = simds.top();
        simds.pop();
        const int s0 = (b.second / kCgpSimds) * kCgpWaves + (b.second % kCgpSimds) * per;   // the SIMD's slots
        int best = s0;
        for (int q = s0 + 1; q < s0 + chainers; ++q)
            if (sload[q] < sload[best]) best = q;
        sload[best] += cost(r);
        lists[best].push_back(r);
        b.first += cost(r);
        simds.push(b);
    }
    std::vector<int> ptr(nwaves + 1, 0), rows;
    rows.reserve(n);
    for (int w = 0; w < nwaves; ++w) {
        std::sort(lists[w].begin(), lists[w].end());
        rows.insert(rows.end(), lists[w].begin(), lists[w].end());
        ptr[w + 1] = (int)rows.size();
    }
    k->wl_ptr = dev_alloc<int>(nwaves + 1);
    k->wl_rows = dev_alloc<int>(n);
    k->tw = dev_alloc<double>(2 * (size_t)n);
    if (!k->wl_ptr || !k->wl_rows || !k->tw ||
        hipMemcpy(k->wl_ptr, ptr.data(), sizeof(int) * (nwaves + 1), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(k->wl_rows, rows.data(), sizeof(int) * n, hipMemcpyHostToDevice) != hipSuccess)
        return;
    k->persist_grid = workers + 1;
}

// SSS_HIP_CG_TRACE: mean phase times (us) of k_cg_persist's iterations 2 .. kCgpTraceIts-1, and the
// workers' SpMV kCgpTraceK, to stderr (diagnostics)
static size_t cg_trace_words(int n, int grid) { return 16 * (size_t)kCgpTraceIts + 4 * (size_t)grid + 5 * (size_t)n; }
static void cg_trace_report(unsigned long long *trc, int n, int grid, const int *rp, hipStream_t s)
{
    std::vector<unsigned long long> h(cg_trace_words(n, grid));
    std::vector<int> hrp(n + 1);
    const bool ok = hipMemcpyAsync(hrp.data(), rp, sizeof(int) * (n + 1), hipMemcpyDeviceToHost, s) == hipSuccess &&
                    hipMemcpyAsync(h.data(), trc, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost, s) ==
                        hipSuccess &&
                    hipStreamSynchronize(s) == hipSuccess;
    (void)hipFree(trc);
    if (!ok) return;
    // relative to iteration k's start (slot 0): t wait done 1, update 2, published 3, norms 4, wave-3 polls 5,
    // all polls 6, t.p chain 7, step 12
    const char *nm[13] = {"period", "t_in", "update", "publish", "norm0", "poll_w3", "poll_all", "tp_chain",
                          "", "", "", "", "step"};
    double acc[13] = {0};
    int cnt = 0;
    for (int k = 2; k + 1 < kCgpTraceIts; ++k) {
        const unsigned long long *a = &h[16 * k], *nx = &h[16 * (k + 1)];
        if (!a[0] || !nx[0] || !a[12]) continue;
        for (int j : {1, 2, 3, 4, 5, 6, 7, 12}) acc[j] += a[j] ? (double)(a[j] - a[0]) * 0.01 : 0.0;
        acc[0] += (double)(nx[0] - a[0]) * 0.01;
        ++cnt;
    }
    std::fprintf(stderr, "[cg trace] %d iterations, us from the iteration's start:", cnt);
    for (int j = 0; j < 13; ++j)
        if (nm[j][0]) std::fprintf(stderr, " %s %.2f", nm[j], cnt ? acc[j] / cnt : 0.0);
    {   // the last run of ready chunks the t.p chain summed in one call: its length and rate
        double len = 0, us = 0;
        int m = 0;
        for (int k = 2; k + 1 < kCgpTraceIts; ++k)
            if (h[16 * k + 8] && h[16 * k + 7] > h[16 * k + 8])
                len += (double)h[16 * k + 9], us += (double)(h[16 * k + 7] - h[16 * k + 8]) * 0.01, ++m;
        if (m) std::fprintf(stderr, " | last chain run: %.0f entries in %.2f us (%.2f ns per entry)", len / m, us / m,
                            len > 0 ? us * 1e3 / len : 0.0);
    }
    std::fprintf(stderr, "\n");
    // SpMV kCgpTraceK, from its (speculative) publish in iteration kCgpTraceK - 1
    const long long P = (long long)h[16 * (kCgpTraceK - 1) + 3];
    const unsigned long long *w = &h[16 * kCgpTraceIts], *r = w + 4 * grid;
    auto rel = [&](unsigned long long t) { return ((long long)t - P) * 0.01; };
    double cmd_lo = 1e30, cmd_hi = -1e30, p_lo = 1e30, p_hi = -1e30;
    for (int b = 1; b < grid; ++b)
        if (w[4 * b])
            cmd_lo = std::min(cmd_lo, rel(w[4 * b])), cmd_hi = std::max(cmd_hi, rel(w[4 * b])),
            p_lo = std::min(p_lo, rel(w[4 * b + 1])), p_hi = std::max(p_hi, rel(w[4 * b + 1]));
    std::vector<int> idx;
    double sdur = 0, slen = 0;
    for (int i = 0; i < n; ++i)
        if (r[4 * i + 1]) idx.push_back(i), sdur += (r[4 * i + 1] - r[4 * i]) * 10.0, slen += hrp[i + 1] - hrp[i];
    std::sort(idx.begin(), idx.end(), [&](int a, int b) { return r[4 * a + 1] > r[4 * b + 1]; });
    std::fprintf(stderr, "[cg trace] SpMV %d from its publish: command %.2f..%.2f, p in LDS %.2f..%.2f; rows %zu, "
                 "%.2f ns per entry; latest rows (row:len start dur [strip loads, chains]):",
                 kCgpTraceK, cmd_lo, cmd_hi, p_lo, p_hi, idx.size(), slen > 0 ? sdur / slen : 0.0);
    for (size_t q = 0; q < 12 && q < idx.size(); ++q) {
        const int i = idx[q];
        std::fprintf(stderr, " %d:%d %.2f %.2f [%.2f %.2f]", i, hrp[i + 1] - hrp[i], rel(r[4 * i]),
                     (r[4 * i + 1] - r[4 * i]) * 0.01, r[4 * i + 2] * 0.01, r[4 * i + 3] * 0.01);
    }
    std::fprintf(stderr, "\n");
    // where the rows ran: per (block, SIMD) the entries chained, against the plan's wave % 4
    std::vector<long long> simd(4 * grid, 0), plan(4 * grid, 0);
    int mism = 0;
    for (int i = 0; i < n; ++i) {
        const unsigned long long x = r[4 * n + i];
        const int gwv = (int)(x >> 32), hw = (int)(x & 0xffff), sm = (hw >> 4) & 3, b = gwv / kCgpWaves;
        simd[4 * b + sm] += hrp[i + 1] - hrp[i];
        plan[4 * b + (gwv % kCgpWaves) / 4] += hrp[i + 1] - hrp[i];
        mism += sm != (gwv % kCgpWaves) / 4;
    }
    std::fprintf(stderr, "[cg trace] rows whose SIMD != plan slot / 4: %d; max entries per SIMD: measured %lld, plan %lld; "
                 "row 0..7 waves/SIMDs:", mism, *std::max_element(simd.begin(), simd.end()),
                 *std::max_element(plan.begin(), plan.end()));
    for (int i = 0; i < 8 && i < n; ++i)
        std::fprintf(stderr, " %d/%d", (int)(r[4 * n + i] >> 32) % kCgpWaves, (int)((r[4 * n + i] >> 4) & 3));
    std::fprintf(stderr, "\n");
}

static int run_cg(CoarseKrylov *k, const DevCSR &A, const double *b, double *u, double tol, int maxit, hipStream_t s,
                  int *status)
{
    const int n = k->n, nblk = A.nblk;
    const char *cr = getenv("SSS_HIP_CG_REG");   // "0": the LDS-chunked step at every size (test hook)
    const bool reg_step = !(cr && cr[0] == '0') && n <= kRegVec * kSeqBlock;
    // the whole loop in one launch (k_cg_persist); SSS_HIP_CG_PERSIST=0: two kernels per iteration (test hook)
    const char *cp = getenv("SSS_HIP_CG_PERSIST");
    const bool persist = reg_step && k->persist_grid > 0 && !(cp && cp[0] == '0');
    int spin = kCgpSpin;
    if (const char *e = getenv("SSS_HIP_CG_SPIN")) spin = atoi(e);
    unsigned long long *trc = nullptr;   // SSS_HIP_CG_TRACE=1: phase timestamps of the first launch (diagnostics)
    static bool traced = false;
    const char *ct = getenv("SSS_HIP_CG_TRACE");
    if (persist && ct && ct[0] == '1' && !traced) {
        traced = true;
        const size_t words = cg_trace_words(n, k->persist_grid);
        if (hipMalloc(&trc, sizeof(unsigned long long) * words) != hipSuccess) trc = nullptr;
        else SSS_HIP(hipMemsetAsync(trc, 0, sizeof(unsigned long long) * words, s));
    }
    SSS_HIP(hipMemsetAsync(k->t, 0, sizeof(double) * n, s));
    SSS_HIP(hipMemsetAsync(k->u_best, 0, sizeof(double) * n, s));
    hipLaunchKernelGGL(k_resid, dim3(nblk), dim3(kBlock), 0, s, A.blk, A.rp, A.ci, A.v, u, b, k->r, k->cap,
                       (const CgState *)nullptr, 0);
    hipLaunchKernelGGL(k_cg_init, dim3(1), dim3(kSeqBlock), 0, s, n, k->r, k->p, tol, maxit, k->st);
    if (persist) {
        k->epoch = (k->epoch + 1) & 0xfffffu;   // 20 bits of launch count above 12 bits of command count
        if (k->epoch == 0) k->epoch = 1;        // (tag 0 is the zeroed granules')
        SSS_HIP(hipMemsetAsync(k->pctl + 64, 0, sizeof(unsigned long long), s));
        hipLaunchKernelGGL(k_cg_persist, dim3(k->persist_grid), dim3(kSeqBlock), 0, s, n, maxit, A.rp, A.ci, A.v, b,
                           k->cap, u, k->r, k->p, k->u_best, k->st, k->gp_p, k->gp_t, k->pctl, k->epoch, k->wl_ptr, k->wl_rows, k->tw, spin, trc);
        SSS_HIP(hipGetLastError());
        if (trc) cg_trace_report(trc, n, k->persist_grid, A.rp, s);
        SSS_HIP(hipMemcpyAsync(k->h_buf + 8, k->pctl + 64, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    }
    for (int it = 1; it <= maxit && !persist; ++it) {
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
    if (persist && reinterpret_cast<const unsigned long long *>(k->h_buf)[8] != 0) {
        fprintf(stderr, "### ERROR: coarse CG: a workgroup of the one-launch CG stalled (spin limit reached); "
                        "the coarse iterate is invalid\n");
        return ERROR_MISC;
    }
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
