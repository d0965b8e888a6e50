/*
 * sss_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker; see sss_oracle.h).
 *
 * A plain-C restatement of the reference solve phase (txthpc/amg, amg/Solve/ and SSS_utils.c),
 * written to reproduce its floating-point results bit for bit when compiled with
 * gcc -O2/-O3 -ffp-contract=off on x86-64:
 *
 *   ora_mv_amxpy / ora_mv_mxy ..... SSS_utils.c:161-201 (row sum from 0.0 in CSR order, then
 *                                    y += sum*alpha / y = sum)
 *   ora_mv_acc .................... Solve/SSS_cuda.cu:77-96 spmv_kernel: y += A*x (accumulates!)
 *   row cap ....................... Solve/SSS_cuda.cu:131,152 <<<64,64>>> -> rows < 4096 only
 *                                    (as-shipped); cap = 0 is the "uncapped" parity definition
 *   ora_gs_cf ..................... Solve/SSS_smooth.c:4-87 (stale d carried across rows)
 *   ora_gs ........................ Solve/SSS_smooth.c:90-137
 *   ora_smoother_pre/post ......... Solve/SSS_smooth.c:138-304
 *   ora_cg ........................ Solve/SSS_cycle.cu:15-437 as compiled: beta == temp1/temp1
 *                                    == 1 and temp1 frozen at (r0,r0),
 *                                    t += A*p accumulates, (z,r) computed and discarded
 *   ora_gmres ..................... Solve/SSS_cycle.cu:440-817 (Arnoldi p[i] += A*r accumulates)
 *   ora_coarest_solve ............. Solve/SSS_cycle.cu:819-846
 *   ora_cycle ..................... Solve/SSS_cycle.cu:848-967
 *   ora_solve ..................... Solve/SSS_SOLVE.c:4-87
 *   ora_interp_std ................ Setup/SSS_inter.cu:550-715 + the truncation, :16-102 (setup;
 *                                    the standard pattern itself is pinned by the compiled
 *                                    SSS_coarsen.c)
 *
 * Only stop_type STOP_REL_RES is restated for the Krylov methods: it is the only one the
 * coarse solver uses (Solve/SSS_cycle.cu:833).
 *
 * Pinning: (1) the reference's pure-C units that build without CUDA
 * (SSS_utils.c, SSS_matvec.c, Solve/SSS_smooth.c, Setup/SSS_coarsen.c, SSS_main.c) are
 * compiled from /root/reference into oracle/_ref/ by oracle/Makefile and compared function by
 * function in tests/test_ref_units.py; (2) the parts that need CUDA headers (cycle, CG/GMRES,
 * interpolation) are pinned by the known-answer tables of SURVEY.md §4 (1138_bus 13-row
 * history, x sums after cycles 1-3 to 17 digits; 16^3 / 32^3 histories), tests/test_oracle.py.
 */
#include "sss_oracle.h"

#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

static double now_s(void)
{
    struct timeval tv;
    gettimeofday(&tv, NULL);
    return (double)tv.tv_sec + (double)tv.tv_usec * 1e-6;
}


/* Local copies of the two reference utilities the solve path prints through, so that the
 * oracle links against nothing from the product (SSS_utils.c:16-133). */
static void ora_print_itinfo(int iter, double relres, double absres, double factor)
{
    if (iter > 0) {
        printf("%6d | %13.6e   | %13.6e  | %10.4lf\n", iter, relres, absres, factor);
        return;
    }
    printf("-----------------------------------------------------------\n");
    printf("It Num |   ||r||/||b||   |     ||r||      |  Conv. Factor\n");
    printf("-----------------------------------------------------------\n");
    printf("%6d | %13.6e   | %13.6e  |     -.-- \n", iter, relres, absres);
}

static void ora_exit_input_par(const char *fname)
{
    printf("### ERROR: %s -- Wrong input arguments!\n", fname);
    exit(ERROR_INPUT_PAR);
}

static double g_coarse_seconds = 0.0;
double ora_coarse_seconds(void) { return g_coarse_seconds; }
void ora_reset_timers(void) { g_coarse_seconds = 0.0; }

void ora_opts_default(ora_opts *o)
{
    memset(o, 0, sizeof(*o));
    o->jacobi_from = 1;
    o->omega = 1.0;
}

/* ---------------------------------------------------------------- BLAS-1, sequential order */
static double dot(int n, const double *x, const double *y)
{
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += x[i] * y[i];
    return s;
}
static double nrm2(int n, const double *x) { return sqrt(dot(n, x, x)); }
static double nrminf(int n, const double *x)
{
    double m = 0.0;
    for (int i = 0; i < n; ++i) {
        double a = x[i] >= 0.0 ? x[i] : -x[i];
        m = m > a ? m : a;
    }
    return m;
}
static void axpy(int n, double a, const double *x, double *y)
{
    for (int i = 0; i < n; ++i) y[i] += a * x[i];
}
static void scal(int n, double a, double *x)
{
    for (int i = 0; i < n; ++i) x[i] *= a;
}
static void copy(int n, const double *x, double *y) { memcpy(y, x, sizeof(double) * (size_t)n); }

/* ---------------------------------------------------------------- SpMV family */
static int capped_rows(int m, int cap) { return (cap > 0 && cap < m) ? cap : m; }

static double row_sum(const SSS_MAT *A, const double *x, int i)
{
    double s = 0.0;
    for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k) s += A->val[k] * x[A->col_idx[k]];
    return s;
}

/* Row loops below may run on several host threads (ora_set_threads; bench.py's multi-core CPU
 * baseline): every row is still summed sequentially in stored order by one thread, so the
 * results do not depend on the thread count. */
void ora_mv_amxpy(double alpha, const SSS_MAT *A, const double *x, double *y, int cap)
{
    const int m = capped_rows(A->num_rows, cap);
#pragma omp parallel for schedule(static, 4096)
    for (int i = 0; i < m; ++i) y[i] += row_sum(A, x, i) * alpha;
}

void ora_mv_mxy(const SSS_MAT *A, const double *x, double *y)
{
#pragma omp parallel for schedule(static, 4096)
    for (int i = 0; i < A->num_rows; ++i) y[i] = row_sum(A, x, i);
}

void ora_mv_acc(const SSS_MAT *A, const double *x, double *y, int cap)
{
    const int m = capped_rows(A->num_rows, cap);
#pragma omp parallel for schedule(static, 4096)
    for (int i = 0; i < m; ++i) y[i] += row_sum(A, x, i);
}

void ora_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }
int ora_get_threads(void) { return omp_get_max_threads(); }

/* ---------------------------------------------------------------- smoothers */
/* one Gauss-Seidel pass over the rows selected by want(mark[i]); d is carried (stale) */
static void gs_pass(double *u, const SSS_MAT *A, const double *b, const int *mark, int c_rows,
                    double *d)
{
    for (int i = 0; i < A->num_rows; ++i) {
        double t;
        if ((mark[i] == 1) != c_rows) continue;
        t = b[i];
        for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k) {
            int j = A->col_idx[k];
            if (j != i) t -= A->val[k] * u[j];
            else *d = A->val[k];
        }
        if ((*d >= 0.0 ? *d : -*d) > SMALLFLOAT) u[i] = t / *d;
    }
}

/* Rows of the class are independent (no same-class off-diagonal entry) and each has exactly one
 * diagonal entry: then the pass gives the same values in any row order (the carried d is always
 * the row's own diagonal), so it may run on several threads.  Cached per (matrix, class). */
static int gs_pass_independent(const SSS_MAT *A, const int *mark, int c_rows)
{
    static struct { const int *ci; const int *mark; int c; int ok; } cache[16];
    static int ncache = 0;
    for (int q = 0; q < ncache; ++q)
        if (cache[q].ci == A->col_idx && cache[q].mark == mark && cache[q].c == c_rows) return cache[q].ok;
    int ok = 1;
#pragma omp parallel for reduction(&& : ok) schedule(static, 4096)
    for (int i = 0; i < A->num_rows; ++i) {
        if ((mark[i] == 1) != c_rows) continue;
        int nd = 0;
        for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k) {
            const int j = A->col_idx[k];
            if (j == i) nd++;
            else if (j < A->num_rows && (mark[j] == 1) == c_rows) ok = 0;
        }
        if (nd != 1) ok = 0;
    }
    if (ncache < 16) cache[ncache].ci = A->col_idx, cache[ncache].mark = mark, cache[ncache].c = c_rows,
                     cache[ncache++].ok = ok;
    return ok;
}

static void gs_pass_any(double *u, const SSS_MAT *A, const double *b, const int *mark, int c_rows, double *d)
{
    if (omp_get_max_threads() == 1 || !gs_pass_independent(A, mark, c_rows)) {
        gs_pass(u, A, b, mark, c_rows, d);
        return;
    }
    const int n = A->num_rows;
#pragma omp parallel for schedule(static, 4096)
    for (int i = 0; i < n; ++i) {
        if ((mark[i] == 1) != c_rows) continue;
        double t = b[i], di = 0.0;
        for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k) {
            const int j = A->col_idx[k];
            if (j != i) t -= A->val[k] * u[j];
            else di = A->val[k];
        }
        if ((di >= 0.0 ? di : -di) > SMALLFLOAT) u[i] = t / di;
    }
    for (int i = n - 1; i >= 0; --i)   /* the divisor register after the pass: the last row's diagonal */
        if ((mark[i] == 1) == c_rows) {
            for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k)
                if (A->col_idx[k] == i) *d = A->val[k];
            break;
        }
}

void ora_gs_cf(double *u, const SSS_MAT *A, const double *b, int sweeps, const int *mark, int order)
{
    double d = 0.0;
    while (sweeps--) {
        gs_pass_any(u, A, b, mark, order ? 0 : 1, &d);
        gs_pass_any(u, A, b, mark, order ? 1 : 0, &d);
    }
}

void ora_gs(double *u, int i1, int in, int step, const SSS_MAT *A, const double *b, int sweeps)
{
    double d = 0.0;
    while (sweeps--) {
        for (int i = i1; step > 0 ? i <= in : i >= in; i += step) {
            double t = b[i];
            for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k) {
                int j = A->col_idx[k];
                if (j != i) t -= A->val[k] * u[j];
                else if (SSS_ABS(A->val[k]) > SMALLFLOAT) d = 1.e+0 / A->val[k];
            }
            u[i] = t * d;
        }
    }
}

/* C/F-Jacobi (engine extension): per sweep an F pass then a C pass; inside a pass
 * every row reads the values from before the pass.  d = last diagonal entry of the row; rows
 * with |d| <= 1e-20 (or none) are left unchanged.  mark == NULL: one pass over all rows. */
void ora_cf_jacobi_w(double *u, const SSS_MAT *A, const double *b, int sweeps, const int *mark, double omega,
                     int l1)
{
    const int n = A->num_rows;
    double *old = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    while (sweeps--) {
        for (int pass = 0; pass < (mark ? 2 : 1); ++pass) {
            copy(n, u, old);
#pragma omp parallel for schedule(static, 4096)
            for (int i = 0; i < n; ++i) {
                double t, d = 0.0, off = 0.0;
                if (mark && (mark[i] == 1) != pass) continue;
                t = b[i];
                for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k) {
                    int j = A->col_idx[k];
                    if (j != i) {
                        t -= A->val[k] * old[j];
                        if (l1 && (!mark || (mark[j] == 1) == pass)) off += SSS_ABS(A->val[k]);
                    } else d = A->val[k];
                }
                if (l1) d += off;
                if (SSS_ABS(d) > SMALLFLOAT) {
                    const double xn = t / d;
                    u[i] = omega == 1.0 ? xn : old[i] + omega * (xn - old[i]);
                }
            }
        }
    }
    free(old);
}

void ora_cf_jacobi(double *u, const SSS_MAT *A, const double *b, int sweeps, const int *mark)
{
    ora_cf_jacobi_w(u, A, b, sweeps, mark, 1.0, 0);
}

/* Two-stage GS-CF (engine extension): each class pass solves the pass's triangular
 * system  (D + L_cc) x_c = b_c - U_cc x_c_old - A_c,other x_other  approximately.  Per row i of the
 * pass, its off-diagonal entries split into L_i (same class, j < i) and N_i (the rest):
 *   P_i  = b_i - sum_{N_i} a_ij x_old_j                    (stored order)
 *   y0_i = (P_i - sum_{L_i} a_ij x_old_j) / d_i            (= the C/F-Jacobi value, other order)
 *   y_s,i = (P_i - sum_{L_i} a_ij y_{s-1},j) / d_i,  s = 1..inner
 * then x_c = y_inner.  P is formed once per pass, so each inner step reads only the L entries.
 * inner >= the pass's DAG depth reproduces ora_gs_cf's values up to that summation order.  d is
 * the row's last diagonal entry; rows with |d| <= 1e-20 keep their value. */
void ora_cf_twostage(double *u, const SSS_MAT *A, const double *b, int sweeps, const int *mark, int inner)
{
    const int n = A->num_rows;
    const size_t sz = sizeof(double) * (size_t)(n > 0 ? n : 1);
    double *old = (double *)malloc(sz), *cur = (double *)malloc(sz), *nxt = (double *)malloc(sz);
    double *P = (double *)malloc(sz), *dg = (double *)malloc(sz);
    while (sweeps--) {
        for (int pass = 0; pass < (mark ? 2 : 1); ++pass) {
#define IN_PASS(r) (!mark || (mark[r] == 1) == pass)
            copy(n, u, old);
            copy(n, u, cur);
#pragma omp parallel for schedule(static, 4096)
            for (int i = 0; i < n; ++i) {   /* P and stage 0 */
                double t, d = 0.0;
                if (!IN_PASS(i)) continue;
                t = b[i];
                for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k) {
                    const int j = A->col_idx[k];
                    if (j == i) d = A->val[k];
                    else if (!(j < i && IN_PASS(j))) t -= A->val[k] * old[j];
                }
                P[i] = t;
                dg[i] = d;
                for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k) {
                    const int j = A->col_idx[k];
                    if (j != i && j < i && IN_PASS(j)) t -= A->val[k] * old[j];
                }
                if (SSS_ABS(d) > SMALLFLOAT) cur[i] = t / d;
            }
            for (int stage = 1; stage <= inner; ++stage) {
                copy(n, cur, nxt);
#pragma omp parallel for schedule(static, 4096)
                for (int i = 0; i < n; ++i) {
                    double t;
                    if (!IN_PASS(i)) continue;
                    t = P[i];
                    for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k) {
                        const int j = A->col_idx[k];
                        if (j != i && j < i && IN_PASS(j)) t -= A->val[k] * cur[j];
                    }
                    if (SSS_ABS(dg[i]) > SMALLFLOAT) nxt[i] = t / dg[i];
                }
                double *sw = cur;
                cur = nxt;
                nxt = sw;
            }
            copy(n, cur, u);
#undef IN_PASS
        }
    }
    free(old);
    free(cur);
    free(nxt);
    free(P);
    free(dg);
}

static const ora_opts *g_cur_opts = NULL;
static int g_cur_level = 0;

static void smoother_dispatch(SSS_SMTR *s, int post, const char *fname)
{
    const int use_cf = s->cf_order && s->ordering != NULL;
    switch (s->smoother) {
    case SSS_SM_GS:
        if (use_cf) ora_gs_cf(s->x->d, s->A, s->b->d, s->nsweeps, s->ordering, post ? -1 : 1);
        else if (!post) ora_gs(s->x->d, s->istart, s->iend, s->istep, s->A, s->b->d, s->nsweeps);
        else ora_gs(s->x->d, s->iend, s->istart, s->istep, s->A, s->b->d, s->nsweeps);
        break;
    case SSS_SM_JACOBI:
        if (g_cur_opts && g_cur_opts->inner > 0 &&
            (!g_cur_opts->inner_mask || (g_cur_opts->inner_mask >> g_cur_level & 1))) {
            const int extra = (g_cur_opts->long_mask >> g_cur_level & 1) ? g_cur_opts->inner_long : 0;
            ora_cf_twostage(s->x->d, s->A, s->b->d, s->nsweeps, use_cf ? s->ordering : NULL, g_cur_opts->inner + extra);
            break;
        }
        ora_cf_jacobi_w(s->x->d, s->A, s->b->d, s->nsweeps, use_cf ? s->ordering : NULL,
                        g_cur_opts ? g_cur_opts->omega : 1.0, g_cur_opts ? g_cur_opts->jacobi_l1 : 0);
        break;
    default:
        printf("### ERROR: Wrong smoother type %d!\n", s->smoother);
        ora_exit_input_par(fname);
    }
}

void ora_smoother_pre(SSS_SMTR *s) { smoother_dispatch(s, 0, "SSS_amg_smoother_pre"); }
void ora_smoother_post(SSS_SMTR *s) { smoother_dispatch(s, 1, "SSS_amg_smoother_post"); }

/* ---------------------------------------------------------------- coarse Krylov */
/* r = b; r += (int)(-1) * A*u   (alpha_spmv_cuda) */
static void residual_into(const SSS_MAT *A, const double *b, const double *u, double *r, int m, int cap)
{
    copy(m, b, r);
    ora_mv_amxpy(-1.0, A, u, r, cap);
}

int ora_cg(SSS_KRYLOV *ks, int cap)
{
    SSS_MAT *A = ks->A;
    const int m = ks->b->n, maxit = ks->matrix;
    const double tol = ks->tol, maxdiff = tol * 1e-4;
    double *u = ks->u->d;
    const double *b = ks->b->d;
    double *work = (double *)calloc(5 * (size_t)m, sizeof(double));
    double *p = work, *z = p + m, *r = z + m, *t = r + m, *u_best = t + m;
    int iter = 0, stag = 1, more_step = 1, iter_best = 0;
    double absres0, absres = BIGFLOAT, relres, normr0, absres_best = BIGFLOAT;
    double alpha, temp1, temp2;

    residual_into(A, b, u, r, m, cap);
    copy(m, r, z);
    absres0 = nrm2(m, r);
    normr0 = SSS_max(SMALLFLOAT, absres0);
    relres = absres0 / normr0;
    if (relres < tol) goto done;
    copy(m, z, p);
    temp1 = dot(m, z, r); /* frozen for the whole solve: Solve/SSS_cycle.cu:373-374 as compiled */

    while (iter++ < maxit) {
        ora_mv_acc(A, p, t, cap);          /* t += A*p: t is never cleared */
        temp2 = dot(m, t, p);
        if (SSS_ABS(temp2) > SMALLFLOAT2) alpha = temp1 / temp2;
        else goto restore;
        axpy(m, alpha, p, u);
        axpy(m, -alpha, t, r);
        absres = nrm2(m, r);
        relres = absres / normr0;
        if (absres < absres_best - maxdiff) {
            absres_best = absres;
            iter_best = iter;
            copy(m, u, u_best);
        }
        if (nrminf(m, u) <= SMALLFLOAT) {
            iter = ERROR_SOLVER_SOLSTAG;
            break;
        }
        {
            const double normu = nrm2(m, u);
            const double reldiff = SSS_ABS(alpha) * nrm2(m, p) / normu;
            if ((stag <= max_STAG) & (reldiff < maxdiff)) {
                residual_into(A, b, u, r, m, cap);
                absres = nrm2(m, r);
                relres = absres / normr0;
                if (relres < tol) break;
                if (stag >= max_STAG) {
                    iter = ERROR_SOLVER_STAG;
                    break;
                }
                memset(p, 0, sizeof(double) * (size_t)m);
                ++stag;
            }
        }
        if (relres < tol) {
            residual_into(A, b, u, r, m, cap);
            absres = nrm2(m, r);
            relres = absres / normr0;
            if (relres < tol) break;
            if (more_step >= max_RESTART) {
                iter = ERROR_SOLVER_TOLSMALL;
                break;
            }
            memset(p, 0, sizeof(double) * (size_t)m);
            ++more_step;
        }
        absres0 = absres;
        copy(m, r, z);
        /* (z,r) is computed and discarded by the reference; beta = temp1/temp1 = 1 */
        for (int i = 0; i < m; ++i) p[i] = 1.0 * z[i] + 1.0 * p[i];
    }

restore:
    if (iter != iter_best) {
        residual_into(A, b, u_best, r, m, cap);
        absres_best = nrm2(m, r);
        if (absres > absres_best + maxdiff) copy(m, u_best, u);
    }
done:
    free(work);
    (void)absres0;
    return iter > maxit ? ERROR_SOLVER_matrix : iter;
}

int ora_gmres(SSS_KRYLOV *ks, int cap)
{
    SSS_MAT *A = ks->A;
    const int n = ks->b->n, maxit = ks->matrix, restart = ks->restart, restart1 = restart + 1;
    const double tol = ks->tol, maxdiff = tol * 1e-4;
    double *x = ks->u->d;
    const double *b = ks->b->d;
    double *work = (double *)calloc((size_t)(restart + 4) * (size_t)(restart + n) + 1, sizeof(double));
    double **p = (double **)calloc((size_t)restart1, sizeof(double *));
    double **hh = (double **)calloc((size_t)restart1, sizeof(double *));
    double *r = work, *w = r + n, *rs = w + n, *c = rs + restart1, *x_best = c + restart, *s = x_best + n;
    double r_norm, t, gamma, normr0, absres = BIGFLOAT, relres, absres_best = BIGFLOAT;
    int iter = 0, iter_best = 0, i = 0;

    for (int q = 0; q < restart1; ++q) p[q] = s + restart + (size_t)q * n;
    for (int q = 0; q < restart1; ++q) hh[q] = p[restart] + n + (size_t)q * restart;

    residual_into(A, b, x, p[0], n, cap);
    r_norm = nrm2(n, p[0]);
    normr0 = SSS_max(SMALLFLOAT, r_norm);
    relres = r_norm / normr0;
    if (relres < tol) goto done;

    while (iter < maxit) {
        rs[0] = r_norm;
        scal(n, 1.0 / r_norm, p[0]);
        i = 0;
        while (i < restart && iter < maxit) {
            i++;
            iter++;
            copy(n, p[i - 1], r);
            ora_mv_acc(A, r, p[i], cap);   /* p[i] += A*r: p[i] keeps old content */
            for (int j = 0; j < i; ++j) {
                hh[j][i - 1] = dot(n, p[j], p[i]);
                axpy(n, -hh[j][i - 1], p[j], p[i]);
            }
            t = nrm2(n, p[i]);
            hh[i][i - 1] = t;
            if (t != 0.0) scal(n, 1.0 / t, p[i]);
            for (int j = 1; j < i; ++j) {
                t = hh[j - 1][i - 1];
                hh[j - 1][i - 1] = s[j - 1] * hh[j][i - 1] + c[j - 1] * t;
                hh[j][i - 1] = -s[j - 1] * t + c[j - 1] * hh[j][i - 1];
            }
            t = hh[i][i - 1] * hh[i][i - 1];
            t += hh[i - 1][i - 1] * hh[i - 1][i - 1];
            gamma = sqrt(t);
            if (gamma == 0.0) gamma = SMALLFLOAT;
            c[i - 1] = hh[i - 1][i - 1] / gamma;
            s[i - 1] = hh[i][i - 1] / gamma;
            rs[i] = -s[i - 1] * rs[i - 1];
            rs[i - 1] = c[i - 1] * rs[i - 1];
            hh[i - 1][i - 1] = s[i - 1] * hh[i][i - 1] + c[i - 1] * hh[i - 1][i - 1];
            absres = r_norm = fabs(rs[i]);
            relres = absres / normr0;
            if (relres <= tol) break;
        }
        /* back substitution and update */
        rs[i - 1] = rs[i - 1] / hh[i - 1][i - 1];
        for (int k = i - 2; k >= 0; k--) {
            t = 0.0;
            for (int j = k + 1; j < i; j++) t -= hh[k][j] * rs[j];
            t += rs[k];
            rs[k] = t / hh[k][k];
        }
        copy(n, p[i - 1], w);
        scal(n, rs[i - 1], w);
        for (int j = i - 2; j >= 0; j--) axpy(n, rs[j], p[j], w);
        copy(n, w, r);
        axpy(n, 1.0, r, x);
        if (absres < absres_best - maxdiff) {
            absres_best = absres;
            iter_best = iter;
            copy(n, x, x_best);
        }
        if (relres <= tol) {
            residual_into(A, b, x, r, n, cap);
            r_norm = nrm2(n, r);
            absres = r_norm;
            relres = absres / normr0;
            if (relres <= tol) break;
            copy(n, r, p[0]);
            i = 0;
        }
        for (int j = i; j > 0; j--) {
            rs[j - 1] = -s[j - 1] * rs[j];
            rs[j] = c[j - 1] * rs[j];
        }
        if (i) axpy(n, rs[i] - 1.0, p[i], p[i]);
        for (int j = i - 1; j > 0; j--) axpy(n, rs[j], p[j], p[i]);
        if (i) {
            axpy(n, rs[0] - 1.0, p[0], p[0]);
            axpy(n, 1.0, p[i], p[0]);
        }
    }

    if (iter != iter_best) {
        residual_into(A, b, x_best, r, n, cap);
        absres_best = nrm2(n, r);
        if (absres > absres_best + maxdiff) copy(n, x_best, x);
    }
done:
    free(work);
    free(p);
    free(hh);
    return iter >= maxit ? ERROR_SOLVER_matrix : iter;
}

/* ---------------------------------------------------------------- direct coarse (LU) */
static struct {
    const void *key;
    int n, nnz;
    double *lu;
    int *piv;
} g_lu;

static void lu_factor(const SSS_MAT *A)
{
    const int n = A->num_rows;
    double *a;
    if (g_lu.key == (const void *)A->val && g_lu.n == n && g_lu.nnz == A->num_nnzs) return;
    free(g_lu.lu);
    free(g_lu.piv);
    a = (double *)calloc((size_t)n * n, sizeof(double));
    g_lu.piv = (int *)malloc(sizeof(int) * (size_t)n);
    for (int i = 0; i < n; ++i)
        for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k) a[(size_t)i * n + A->col_idx[k]] += A->val[k];
    for (int k = 0; k < n; ++k) {
        int pr = k;
        double best = fabs(a[(size_t)k * n + k]);
        for (int i = k + 1; i < n; ++i)
            if (fabs(a[(size_t)i * n + k]) > best) { best = fabs(a[(size_t)i * n + k]); pr = i; }
        g_lu.piv[k] = pr;
        if (pr != k)
            for (int j = 0; j < n; ++j) {
                double tmp = a[(size_t)k * n + j];
                a[(size_t)k * n + j] = a[(size_t)pr * n + j];
                a[(size_t)pr * n + j] = tmp;
            }
        if (a[(size_t)k * n + k] == 0.0) continue;
#pragma omp parallel for schedule(static, 16)
        for (int i = k + 1; i < n; ++i) {
            double f = a[(size_t)i * n + k] / a[(size_t)k * n + k];
            a[(size_t)i * n + k] = f;
            if (f != 0.0)
                for (int j = k + 1; j < n; ++j) a[(size_t)i * n + j] -= f * a[(size_t)k * n + j];
        }
    }
    g_lu.lu = a;
    g_lu.key = A->val;
    g_lu.n = n;
    g_lu.nnz = A->num_nnzs;
}

static void lu_solve(const SSS_MAT *A, const double *b, double *x)
{
    const int n = A->num_rows;
    lu_factor(A);
    copy(n, b, x);
    for (int k = 0; k < n; ++k) {
        int pr = g_lu.piv[k];
        if (pr != k) { double tmp = x[k]; x[k] = x[pr]; x[pr] = tmp; }
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j) x[i] -= g_lu.lu[(size_t)i * n + j] * x[j];
    for (int i = n - 1; i >= 0; --i) {
        for (int j = i + 1; j < n; ++j) x[i] -= g_lu.lu[(size_t)i * n + j] * x[j];
        x[i] /= g_lu.lu[(size_t)i * n + i];
    }
}

void ora_coarest_solve(SSS_MAT *A, SSS_VEC *b, SSS_VEC *x, double ctol, const ora_opts *o)
{
    const int n = A->num_rows;
    const int nn = (int)(int32_t)((int64_t)n * n);   /* n*n in int, as the reference */
    const double t0 = now_s();
    SSS_KRYLOV ks;
    int status;

    if (o && o->coarse_mode == 1) {
        lu_solve(A, b->d, x->d);
        g_coarse_seconds += now_s() - t0;
        return;
    }
    ks.A = A;
    ks.b = b;
    ks.u = x;
    ks.tol = ctol;
    ks.matrix = SSS_max(250, SSS_MIN(nn, 1000));
    ks.stop_type = STOP_REL_RES;
    ks.restart = max_RESTART;
    status = ora_cg(&ks, o ? o->row_cap : 0);
    if (status < 0) {
        ks.restart = max_RESTART;
        status = ora_gmres(&ks, o ? o->row_cap : 0);
    }
    if (status < 0 && (!o || o->verbose)) printf("### WARNING: Coarse level solver failed to converge!\n");
    g_coarse_seconds += now_s() - t0;
}

/* ---------------------------------------------------------------- V/W cycle */
static void level_smoother(SSS_AMG *mg, int l, int post, const ora_opts *o)
{
    SSS_SMTR s;
    memset(&s, 0, sizeof(s));
    s.smoother = mg->pars.smoother;
    if (o && o->smoother == 1 && l >= o->jacobi_from) s.smoother = SSS_SM_JACOBI;
    s.A = &mg->cg[l].A;
    s.b = &mg->cg[l].b;
    s.x = &mg->cg[l].x;
    s.nsweeps = post ? mg->pars.post_iter : mg->pars.pre_iter;
    s.istart = 0;
    s.iend = mg->cg[l].A.num_rows - 1;
    s.istep = post ? -1 : 1;
    s.relax = mg->pars.relax;
    s.ndeg = mg->pars.poly_deg;
    s.cf_order = mg->pars.cf_order;
    s.ordering = mg->cg[l].cfmark.d;
    g_cur_opts = o;
    g_cur_level = l;
    if (post) ora_smoother_post(&s);
    else ora_smoother_pre(&s);
    g_cur_opts = NULL;
}

void ora_cycle(SSS_AMG *mg, const ora_opts *o)
{
    const int nl = mg->num_levels;
    int cycle_type = mg->pars.cycle_type;
    double tol = mg->pars.ctol;
    int visits[max_AMG_LVL] = {0};
    int l = 0;

    if (tol > mg->pars.tol) tol = mg->pars.tol * 0.1;
    if (cycle_type <= 0) cycle_type = 1;
    for (;;) {
        while (l < nl - 1) {
            SSS_AMG_COMP *L = &mg->cg[l];
            visits[l]++;
            level_smoother(mg, l, 0, o);
            copy(L->A.num_rows, L->b.d, L->wp.d);
            ora_mv_amxpy(-1.0, &L->A, L->x.d, L->wp.d, 0);
            ora_mv_mxy(&L->R, L->wp.d, mg->cg[l + 1].b.d);
            l++;
            memset(mg->cg[l].x.d, 0, sizeof(double) * (size_t)mg->cg[l].x.n);
        }
        ora_coarest_solve(&mg->cg[nl - 1].A, &mg->cg[nl - 1].b, &mg->cg[nl - 1].x, tol, o);
        while (l > 0) {
            l--;
            ora_mv_amxpy(1.0, &mg->cg[l].P, mg->cg[l + 1].x.d, mg->cg[l].x.d, 0);
            level_smoother(mg, l, 1, o);
            if (visits[l] < cycle_type) break;
            visits[l] = 0;
        }
        if (l <= 0) break;
    }
}

/* ---------------------------------------------------------------- outer loop */
SSS_RTN ora_solve(SSS_AMG *mg, SSS_VEC *x, SSS_VEC *b, const ora_opts *o, double *relres_hist,
                  double *absres_hist, int hist_cap)
{
    const int verbose = o ? o->verbose : 0;
    const SSS_MAT *A0 = &mg->cg[0].A;
    double *r = mg->cg[0].wp.d;
    const double sumb = nrm2(b->n, b->d);
    double absres0 = sumb, t0 = now_s();
    SSS_RTN rtn = {0.0, 0.0, 0};

    if (verbose) ora_print_itinfo(0, 1.0, sumb, 0.0);
    if (fabs(sumb) == 0.0) {
        memset(x->d, 0, sizeof(double) * (size_t)x->n);
        mg->rtn = rtn;
        return rtn;
    }
    mg->cg[0].x = *x;
    mg->cg[0].b = *b;
    for (int iter = 1; iter <= mg->pars.max_it; ++iter) {
        double absres, relres, factor;
        ora_cycle(mg, o);
        copy(b->n, b->d, r);
        ora_mv_amxpy(-1.0, A0, x->d, r, 0);
        absres = nrm2(b->n, r);
        relres = absres / sumb;
        factor = absres / absres0;
        absres0 = absres;
        if (verbose) ora_print_itinfo(iter, relres, absres, factor);
        if (iter <= hist_cap) {
            if (relres_hist) relres_hist[iter - 1] = relres;
            if (absres_hist) absres_hist[iter - 1] = absres;
        }
        rtn.ares = absres;
        rtn.rres = relres;
        rtn.nits = iter;
        mg->rtn = rtn;
        if (relres < mg->pars.tol) break;
    }
    if (verbose) printf("AMG solve time: %g s\n", now_s() - t0);
    return rtn;
}

/* ---------------------------------------------------------------------------------------------
 * Setup/SSS_inter.cu:16-102: per row, keep entries >= eps * (largest positive) or <= eps *
 * (smallest negative), rescale the kept positives / negatives to the row's full sums.
 * ------------------------------------------------------------------------------------------- */
static void ora_interp_trunc(SSS_MAT *P, double eps)
{
    int nz = 0, w1 = 0, w2 = 0;
    for (int i = 0; i < P->num_rows; ++i) {
        const int lo = P->row_ptr[i], hi = P->row_ptr[i + 1];
        double mneg = 0, mpos = 0, sneg = 0, spos = 0, tneg = 0, tpos = 0;
        P->row_ptr[i] = nz;
        for (int j = lo; j < hi; ++j) {
            if (P->val[j] > 0) {
                spos += P->val[j];
                mpos = mpos > P->val[j] ? mpos : P->val[j];
            } else if (P->val[j] < 0) {
                sneg += P->val[j];
                mneg = mneg < P->val[j] ? mneg : P->val[j];
            }
        }
        mpos *= eps;
        mneg *= eps;
        for (int j = lo; j < hi; ++j) {
            if (P->val[j] >= mpos) {
                nz++;
                P->col_idx[w1++] = P->col_idx[j];
                tpos += P->val[j];
            } else if (P->val[j] <= mneg) {
                nz++;
                P->col_idx[w1++] = P->col_idx[j];
                tneg += P->val[j];
            }
        }
        const double fpos = tpos > SMALLFLOAT ? spos / tpos : 1.0;
        const double fneg = tneg < -SMALLFLOAT ? sneg / tneg : 1.0;
        for (int j = lo; j < hi; ++j) {
            if (P->val[j] >= mpos) P->val[w2++] = P->val[j] * fpos;
            else if (P->val[j] <= mneg) P->val[w2++] = P->val[j] * fneg;
        }
    }
    P->num_nnzs = P->row_ptr[P->num_rows] = nz;
}

/* Setup/SSS_inter.cu:550-715, the reference's row loop with its shared scratch arrays. */
void ora_interp_std(const SSS_MAT *A, const int *mark, SSS_MAT *P, const SSS_IMAT *S, double trunc)
{
    const int n = A->num_rows;
    const size_t m = (size_t)(n > 0 ? n : 1);
    int *cindex = malloc(sizeof(int) * m), *rindi = malloc(sizeof(int) * 2 * m), *rindk = malloc(sizeof(int) * 2 * m);
    double *csum = calloc(m, sizeof(double)), *psum = calloc(m, sizeof(double)), *nsum = calloc(m, sizeof(double));
    double *diag = calloc(m, sizeof(double)), *ahat = calloc(m, sizeof(double));
    double alpha = 0.0;
    for (int i = 0; i < n; ++i) cindex[i] = -1;
    /* step 0 (SSS_inter.cu:587-614) */
    for (int i = 0; i < n; ++i) {
        for (int j = S->row_ptr[i]; j < S->row_ptr[i + 1]; ++j)
            if (mark[S->col_idx[j]] == CGPT) cindex[S->col_idx[j]] = i;
        for (int j = A->row_ptr[i]; j < A->row_ptr[i + 1]; ++j) {
            const int k = A->col_idx[j];
            if (cindex[k] == i) csum[i] += A->val[j];
            if (k == i) {
                diag[i] = A->val[j];
            } else {
                nsum[i] += A->val[j];
                if (mark[k] != ISPT) psum[i] += A->val[j];
            }
        }
    }
    /* step 1 (:616-687) */
    for (int i = 0; i < n; ++i) {
        if (mark[i] == FGPT) {
            double alN = psum[i], alP = csum[i];
            for (int j = A->row_ptr[i]; j < A->row_ptr[i + 1]; ++j) rindi[A->col_idx[j]] = j;
            for (int j = P->row_ptr[i]; j < P->row_ptr[i + 1]; ++j) ahat[P->col_idx[j]] = 0.0;
            ahat[i] = diag[i];
            for (int j = S->row_ptr[i]; j < S->row_ptr[i + 1]; ++j) {
                const int k = S->col_idx[j];
                const double aik = A->val[rindi[k]];
                if (mark[k] == CGPT) {
                    ahat[k] += aik;
                } else if (mark[k] == FGPT) {
                    const double akk = diag[k];
                    double aki = 0.0, factor;
                    for (int q = A->row_ptr[k]; q < A->row_ptr[k + 1]; ++q) rindk[A->col_idx[q]] = q;
                    factor = aik / akk;
                    for (int q = A->row_ptr[k]; q < A->row_ptr[k + 1]; ++q)
                        if (A->col_idx[q] == i) {
                            aki = A->val[q];
                            ahat[i] -= factor * aki;
                        }
                    for (int q = S->row_ptr[k]; q < S->row_ptr[k + 1]; ++q) {
                        const int l = S->col_idx[q];
                        const double akl = A->val[rindk[l]];
                        if (mark[l] == CGPT) ahat[l] -= factor * akl;
                    }
                    alN -= factor * (nsum[k] - aki + akk);
                    alP -= factor * csum[k];
                }
            }
            if (P->row_ptr[i + 1] > P->row_ptr[i]) alpha = alN / alP;
            for (int j = P->row_ptr[i]; j < P->row_ptr[i + 1]; ++j) {
                const int k = P->col_idx[j];
                P->val[j] = -alpha * ahat[k] / ahat[i];
            }
        } else if (mark[i] == CGPT) {
            P->val[P->row_ptr[i]] = 1.0;
        }
    }
    /* step 2 (:689-700) */
    int index = 0;
    for (int i = 0; i < n; ++i)
        if (mark[i] == CGPT) cindex[i] = index++;
    P->num_cols = index;
    for (int q = 0; q < P->row_ptr[P->num_rows]; ++q) P->col_idx[q] = cindex[P->col_idx[q]];
    free(cindex), free(rindi), free(rindk), free(csum), free(psum), free(nsum), free(diag), free(ahat);
    /* step 3 (:713-714) */
    ora_interp_trunc(P, trunc);
}
