/*
 * sss_amg.h — drop-in C ABI of the MI355X AMG solve-phase engine.
 *
 * This header is the boundary a user of the txthpc/amg reference links against instead of
 * SSS_AMG.h / SSS_main.h / SSS_utils.h / SSS_matvec.h / Solve/ headers / Setup/SSS_SETUP.h.
 * Every struct keeps the reference's field order and therefore its x86-64 LP64 layout
 * (sizes checked by tests/test_abi.py against SURVEY.md §8b); every function keeps the
 * reference's name, argument meaning and (exit-on-error) behaviour.  Paths below are relative
 * to the reference tree (amg/).
 *
 * What runs where:
 *   - SSS_amg_solve / SSS_amg_cycle / SSS_amg_coarest_solve / SSS_amg_smoother_pre|post /
 *     SSS_blas_mv_amxpy / SSS_blas_mv_mxy run on the GPU (hand-written gfx950 HIP kernels in
 *     libsss_amg.so).  They fail loudly (exit(ERROR_MISC)) when no HIP device is usable.
 *   - Setup (coarsening, interpolation, R = P^T, RAP), .mtx ingest and the small host
 *     utilities stay host C, exactly as in the reference (SURVEY.md §1 L2a is out of scope).
 */
#ifndef SSS_AMG_MI355X_H
#define SSS_AMG_MI355X_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants: SSS_main.h:13-34 ---------------------------------------------------- */
#define TRUE 1
#define FALSE 0
#define max_AMG_LVL 30
#define max_STAG 20
#define max_RESTART 30
#define BIGFLOAT 1e+20
#define SMALLFLOAT2 1e-40
#define SMALLFLOAT 1e-20
#define LIST_HEAD -1
#define LIST_TAIL -2
#define FGPT 0
#define CGPT 1
#define ISPT 2
#define UNPT -1
#define MIN_CDOF 10
#define SSS_max(a, b) (((a) > (b)) ? (a) : (b))
#define SSS_MIN(a, b) (((a) < (b)) ? (a) : (b))
#define SSS_ABS(a) (((a) >= 0.0) ? (a) : -(a))

/* ---- error codes: SSS_main.h:37-63 ---------------------------------------------------- */
typedef enum {
    ERROR_OPEN_FILE = -10,
    ERROR_WRONG_FILE = -11,
    ERROR_INPUT_PAR = -12,
    ERROR_MAT_SIZE = -13,
    ERROR_MISC = -14,
    ERROR_ALLOC_MEM = -20,
    ERROR_DATA_STRUCTURE = -21,
    ERROR_DATA_ZERODIAG = -22,
    ERROR_DUMMY_VAR = -23,
    ERROR_AMG_interp_type = -30,
    ERROR_AMG_SMOOTH_TYPE = -31,
    ERROR_AMG_COARSE_TYPE = -32,
    ERROR_AMG_COARSEING = -33,
    ERROR_SOLVER_STAG = -42,
    ERROR_SOLVER_SOLSTAG = -43,
    ERROR_SOLVER_TOLSMALL = -44,
    ERROR_SOLVER_matrix = -48,
    ERROR_SOLVER_EXIT = -49,
    ERROR_UNKNOWN = -99
} SSS_ERROR_CODE;

/* SSS_main.h:87-93 */
typedef enum { STOP_REL_RES = 1, STOP_REL_PRECRES = 2, STOP_MOD_REL_RES = 3 } SSS_STOP_TYPE;

/* ---- data types (layout-identical to SSS_main.h:95-251) ------------------------------- */
typedef struct SSS_MAT_ {          /* CSR, SSS_main.h:95-105; sizeof 40 */
    int num_rows;
    int num_cols;
    int num_nnzs;
    int *row_ptr;
    int *col_idx;
    double *val;
} SSS_MAT;

typedef struct SSS_IMAT_ {         /* SSS_main.h:107-117 */
    int num_rows;
    int num_cols;
    int num_nnzs;
    int *row_ptr;
    int *col_idx;
    int *val;
} SSS_IMAT;

typedef struct SSS_VEC_ {          /* SSS_main.h:119-124; sizeof 16 */
    int n;
    double *d;
} SSS_VEC;

typedef struct SSS_IVEC_ {         /* SSS_main.h:126-131 */
    int n;
    int *d;
} SSS_IVEC;

typedef enum SSS_SM_TYPE_ {        /* SSS_main.h:133-145 */
    SSS_SM_JACOBI = 1,
    SSS_SM_GS = 2,
    SSS_SM_SGS = 3,
    SSS_SM_SOR = 4,
    SSS_SM_SSOR = 5,
    SSS_SM_GSOR = 6,
    SSS_SM_SGSOR = 7,
    SSS_SM_POLY = 8,
    SSS_SM_L1DIAG = 9
} SSS_SM_TYPE;

typedef enum interp_type_ { intERP_DIR = 1, intERP_STD = 2 } interp_type;   /* SSS_main.h:147-152 */

typedef struct SSS_RTN_ {          /* SSS_main.h:154-160; sizeof 24 */
    double ares;
    double rres;
    int nits;
} SSS_RTN;

typedef enum SSS_COARSEN_TYPE_ { SSS_COARSE_RS = 1, SSS_COARSE_RSP = 2 } SSS_COARSEN_TYPE;

typedef struct SSS_AMG_PARS_ {     /* SSS_main.h:170-194; sizeof 104 */
    int cycle_type;
    double tol;
    double ctol;
    int max_it;
    SSS_COARSEN_TYPE cs_type;
    int max_levels;
    int coarse_dof;
    SSS_SM_TYPE smoother;
    double relax;
    int cf_order;
    int pre_iter;
    int post_iter;
    int poly_deg;
    interp_type interp_type;
    double strong_threshold;
    double max_row_sum;
    double trunc_threshold;
} SSS_AMG_PARS;

typedef struct SSS_AMG_COMP_ {     /* SSS_main.h:196-207; sizeof 184 */
    SSS_MAT A;
    SSS_MAT R;
    SSS_MAT P;
    SSS_VEC b;
    SSS_VEC x;
    SSS_IVEC cfmark;
    SSS_VEC wp;
} SSS_AMG_COMP;

typedef struct SSS_AMG {           /* SSS_main.h:209-218; sizeof 144 */
    int num_levels;
    SSS_AMG_COMP *cg;
    SSS_AMG_PARS pars;
    SSS_RTN rtn;
} SSS_AMG;

typedef struct SSS_SMTR_ {         /* SSS_main.h:221-238; sizeof 72 */
    SSS_SM_TYPE smoother;
    SSS_MAT *A;
    SSS_VEC *b;
    SSS_VEC *x;
    double relax;
    int nsweeps;
    int istart;
    int iend;
    int istep;
    int ndeg;
    int cf_order;
    int *ordering;
} SSS_SMTR;

typedef struct SSS_KRYLOV_ {       /* SSS_main.h:241-251; sizeof 48 */
    double tol;
    SSS_MAT *A;
    SSS_VEC *b;
    SSS_VEC *u;
    int restart;
    int matrix;
    int stop_type;
} SSS_KRYLOV;

/* ======================================================================================
 * Solve phase — the hot path (GPU).  Replaces Solve/SSS_SOLVE.h, Solve/SSS_cycle.h,
 * Solve/SSS_smooth.h and the SpMV half of SSS_utils.h.
 * ====================================================================================== */

/* Solve/SSS_SOLVE.h:9 (Solve/SSS_SOLVE.c:4-87).  Outer loop: V-cycle, r = b - A0 x, ||r||,
 * print, stop on ||r||/||b|| < tol.  The hierarchy is mirrored to HBM on the first call
 * (keyed by mg->cg) and x is written back to x->d before return. */
SSS_RTN SSS_amg_solve(SSS_AMG *mg, SSS_VEC *x, SSS_VEC *b);

/* Solve/SSS_cycle.h:19 (Solve/SSS_cycle.cu:848-967).  One V- (or W-) cycle on the level
 * vectors held in mg; host state is synchronised back before return. */
void SSS_amg_cycle(SSS_AMG *mg);

/* Solve/SSS_cycle.h:17 (Solve/SSS_cycle.cu:819-846).  Coarsest-grid CG(+GMRES) solve. */
void SSS_amg_coarest_solve(SSS_MAT *A, SSS_VEC *b, SSS_VEC *x, const double ctol);

/* Solve/SSS_smooth.h:18-20 (Solve/SSS_smooth.c:138-304).  Gauss-Seidel smoothers. */
void SSS_amg_smoother_pre(SSS_SMTR *s);
void SSS_amg_smoother_post(SSS_SMTR *s);

/* SSS_utils.h:27,30 (SSS_utils.c:161-201).  y += alpha*A*x and y = A*x. */
void SSS_blas_mv_amxpy(double alpha, const SSS_MAT *A, const SSS_VEC *x, SSS_VEC *y);
void SSS_blas_mv_mxy(const SSS_MAT *A, const SSS_VEC *x, SSS_VEC *y);

/* SSS_AMG.h:12 (SSS_AMG.c:9-61).  setup + solve + destroy. */
SSS_RTN SSS_solver_amg(SSS_MAT *A, SSS_VEC *x, SSS_VEC *b, SSS_AMG_PARS *pars);

/* ======================================================================================
 * Host utilities (SSS_utils.h:11-47, SSS_matvec.h:12-69) — host C, as in the reference.
 * ====================================================================================== */
double SSS_get_time(void);
void SSS_free(void *mem);
double SSS_blas_vec_norm2(const SSS_VEC *x);
void SSS_print_itinfo(const int stop_type, const int iter, const double relres,
                      const double absres, const double factor);
void SSS_exit_on_errcode(const int status, const char *fctname);
double SSS_blas_array_norm2(int n, const double *x);
double SSS_blas_array_dot(int n, const double *x, const double *y);
void SSS_blas_array_axpy(int n, double a, const double *x, double *y);
double SSS_blas_array_norminf(int n, const double *x);
void SSS_blas_array_set(int n, double *x, double Ax);
void SSS_blas_array_axpby(int n, double a, const double *x, double b, double *y);
void SSS_blas_array_ax(int n, double a, double *x);

SSS_VEC SSS_vec_create(int m);
void SSS_vec_set_value(SSS_VEC *x, double Ax);
void SSS_mat_destroy(SSS_MAT *A);
void SSS_vec_destroy(SSS_VEC *u);
void *SSS_calloc(size_t size, int type);
SSS_AMG SSS_amg_data_create(SSS_AMG_PARS *pars);
SSS_IVEC SSS_ivec_create(int m);
SSS_MAT SSS_mat_struct_create(int m, int n, int nnz);
void SSS_vec_cp(const SSS_VEC *x, SSS_VEC *y);
void SSS_iarray_cp(const int n, int *x, int *y);
void SSS_blas_array_cp(int n, const double *x, double *y);
void SSS_mat_cp(SSS_MAT *src, SSS_MAT *des);
SSS_VEC SSS_mat_get_diag(SSS_MAT *A, int n);
void SSS_ivec_destroy(SSS_IVEC *u);
/* SSS_matvec.c:202-228; additionally releases the HBM mirror of mg (if any). */
void SSS_amg_data_destroy(SSS_AMG *mg);
SSS_IMAT SSS_imat_trans(SSS_IMAT *A);
void SSS_iarray_set(const int n, int *x, const int Ax);
void SSS_imat_destroy(SSS_IMAT *A);
SSS_MAT SSS_mat_trans(SSS_MAT *A);
SSS_MAT SSS_blas_mat_rap(const SSS_MAT *R, const SSS_MAT *A, const SSS_MAT *P);
void *SSS_realloc(void *oldmem, size_t tsize);

/* ======================================================================================
 * Setup (host C; Setup/SSS_SETUP.h:15-17, Setup/SSS_coarsen.h:41, Setup/SSS_inter.h:64-72).
 * Semantics are the "uncapped" reference: interp_DIR's host arithmetic.
 * ====================================================================================== */
void SSS_amg_complexity_print(SSS_AMG *mg);
void SSS_amg_setup(SSS_AMG *mg, SSS_MAT *A, SSS_AMG_PARS *pars);
int SSS_amg_coarsen(SSS_MAT *A, SSS_IVEC *vertices, SSS_MAT *P, SSS_IMAT *S, SSS_AMG_PARS *pars);
void SSS_amg_interp(SSS_MAT *A, SSS_IVEC *vertices, SSS_MAT *P, SSS_IMAT *S, SSS_AMG_PARS *pars);
void SSS_amg_interp_trunc(SSS_MAT *P, SSS_AMG_PARS *pars);
void interp_DIR(SSS_MAT *A, SSS_IVEC *vertices, SSS_MAT *P, SSS_AMG_PARS *pars);

/* ======================================================================================
 * CLI-side entry points (SSS_main.c:12-119) and .mtx ingest (mmio_highlevel.h:10-305).
 * ====================================================================================== */
void SSS_mat_read(char *filemat, SSS_MAT *A);
void SSS_amg_pars_init(SSS_AMG_PARS *pars);
void SSS_amg_pars_print(SSS_AMG_PARS *pars);
int mmio_info(int *m, int *n, int *nnz, int *isSymmetric, char *filename);
int mmio_data(int *csrRowPtr, int *csrColIdx, double *csrAx, char *filename);

#ifdef __cplusplus
}
#endif

#endif /* SSS_AMG_MI355X_H */
