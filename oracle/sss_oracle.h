/*
 * sss_oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference solve phase,
 * used as the parity checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg.  Never linked into or called by the product (libsss_amg.so).
 *
 * Parity pinning: see oracle/sss_oracle.c header.
 */
#ifndef SSS_ORACLE_H
#define SSS_ORACLE_H

#include "../include/sss_amg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int row_cap;      /* 0: uncapped coarse SpMV (parity definition); 4096: as-shipped <<<64,64>>> */
    int coarse_mode;  /* 0: reference CG(beta==1)+GMRES(30); 1: dense LU direct solve */
    int smoother;     /* 0: exact smoother per pars (GS-CF); 1: C/F-Jacobi on levels >= jacobi_from */
    int jacobi_from;  /* first level that uses C/F-Jacobi when smoother == 1 */
    int verbose;      /* print the reference iteration table */
    int jacobi_l1;    /* C/F-Jacobi divisor: 0 = a_ii, 1 = a_ii + sum_{j != i} |a_ij| over same-class j (l1) */
    double omega;     /* C/F-Jacobi weight (1.0 = plain) */
    int inner;        /* > 0: two-stage GS-CF instead of C/F-Jacobi, with `inner` Jacobi-Richardson
                         steps on the same-class lower triangle (ora_cf_twostage) */
    int inner_mask;   /* experiments: bit l set = level l uses two-stage (0 = every C/F-Jacobi level) */
    int inner_long;   /* extra inner steps on the two-stage levels whose bit is set in long_mask (the
                         engine's long-row levels, sss_hip_opts::inner_long) */
    int long_mask;
} ora_opts;

void ora_opts_default(ora_opts *o);

/* SSS_utils.c:161-201 (+ the row cap of Solve/SSS_cuda.cu:131,152 when cap > 0) */
/* host threads for the row-parallel loops (results do not depend on it) */
void ora_set_threads(int n);
int ora_get_threads(void);
void ora_mv_amxpy(double alpha, const SSS_MAT *A, const double *x, double *y, int cap);
void ora_mv_mxy(const SSS_MAT *A, const double *x, double *y);
void ora_mv_acc(const SSS_MAT *A, const double *x, double *y, int cap);

/* Solve/SSS_smooth.c */
void ora_gs_cf(double *u, const SSS_MAT *A, const double *b, int sweeps, const int *mark, int order);
void ora_gs(double *u, int i1, int in, int step, const SSS_MAT *A, const double *b, int sweeps);
void ora_cf_jacobi(double *u, const SSS_MAT *A, const double *b, int sweeps, const int *mark);
void ora_cf_jacobi_w(double *u, const SSS_MAT *A, const double *b, int sweeps, const int *mark, double omega,
                     int l1);
void ora_cf_twostage(double *u, const SSS_MAT *A, const double *b, int sweeps, const int *mark, int inner);
void ora_smoother_pre(SSS_SMTR *s);
void ora_smoother_post(SSS_SMTR *s);

/* Solve/SSS_cycle.cu */
int ora_cg(SSS_KRYLOV *ks, int cap);
int ora_gmres(SSS_KRYLOV *ks, int cap);
void ora_coarest_solve(SSS_MAT *A, SSS_VEC *b, SSS_VEC *x, double ctol, const ora_opts *o);
void ora_cycle(SSS_AMG *mg, const ora_opts *o);

/* Solve/SSS_SOLVE.c:4-87; relres/absres of iterations 1..nits are stored (if non-NULL) */
SSS_RTN ora_solve(SSS_AMG *mg, SSS_VEC *x, SSS_VEC *b, const ora_opts *o, double *relres_hist,
                  double *absres_hist, int hist_cap);

/* Setup/SSS_inter.cu:550-715 (interp_STD) + :16-102 (SSS_amg_interp_trunc), sequential: fills the
 * values of the standard-interpolation pattern P (fine column indices, as SSS_amg_coarsen returns
 * it), renumbers its columns to coarse indices and truncates with `trunc`. */
void ora_interp_std(const SSS_MAT *A, const int *mark, SSS_MAT *P, const SSS_IMAT *S, double trunc);

/* Seconds spent inside ora_coarest_solve since the last reset (baseline split). */
double ora_coarse_seconds(void);
void ora_reset_timers(void);

#ifdef __cplusplus
}
#endif
#endif
