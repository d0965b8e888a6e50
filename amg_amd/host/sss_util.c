/*
 * sss_util.c — host-side utilities of the drop-in ABI: timers, error exit, iteration printer,
 * vector/matrix lifetime helpers and the host BLAS-1 helpers that setup and the CLI use.
 *
 * Behavioural sources (reference tree amg/):
 *   SSS_utils.c:3-12 (timer), :16-94 (error exit), :104-133 (iteration table), :138-260 (BLAS-1)
 *   SSS_matvec.c:3-228 (allocation, copies, data create/destroy), :247-387 (transposes)
 * The SpMV entry points SSS_blas_mv_amxpy / _mxy are NOT here: they are GPU-backed
 * (amg_amd/host/sss_solve.c).
 */
#include "sss_internal.h"

struct hsa_agent_s;   /* (named in roctx.h's prototypes; declared here so C sees one type) */
struct ihipStream_t;
#include <rocprofiler-sdk-roctx/roctx.h>
#include <stdarg.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <sys/mman.h>
#include <sys/time.h>
#include <stdint.h>

#include <omp.h>

double SSS_get_time(void)
{
    struct timeval now;
    gettimeofday(&now, NULL);
    return (double)now.tv_sec + (double)now.tv_usec * 1e-6;
}

void SSS_free(void *mem)
{
    free(mem);
}

/* Message table of SSS_utils.c:20-91.  Codes without a message only exit. */
static const char *errcode_message(int status)
{
    switch (status) {
    case ERROR_OPEN_FILE: return "Cannot open file!";
    case ERROR_WRONG_FILE: return "Wrong file format!";
    case ERROR_INPUT_PAR: return "Wrong input arguments!";
    case ERROR_ALLOC_MEM: return "Cannot allocate memory!";
    case ERROR_DATA_STRUCTURE: return "Data structure mismatch!";
    case ERROR_DATA_ZERODIAG: return "Matrix has zero diagonal entries!";
    case ERROR_DUMMY_VAR: return "Unexpected input argument!";
    case ERROR_AMG_interp_type: return "Unknown AMG interPolation type!";
    case ERROR_AMG_COARSE_TYPE: return "Unknown AMG coarsening type!";
    case ERROR_AMG_SMOOTH_TYPE: return "Unknown AMG smoother type!";
    case ERROR_SOLVER_STAG: return "Solver stagnation error!";
    case ERROR_SOLVER_SOLSTAG: return "Solution is close to zero!";
    case ERROR_SOLVER_TOLSMALL: return "Tol is too small for the solver!";
    case ERROR_SOLVER_matrix: return "max iteration number reached!";
    case ERROR_SOLVER_EXIT: return "Solver exited unexpected!";
    case ERROR_MISC: return "Unknown error occurred!";
    case ERROR_UNKNOWN: return "Function does not exit successfully!";
    default: return NULL;
    }
}

void SSS_exit_on_errcode(const int status, const char *fctname)
{
    const char *msg;
    if (status >= 0) return;
    msg = errcode_message(status);
    if (msg) printf("### ERROR: %s -- %s\n", fctname, msg);
    exit(status);
}

/* SSS_utils.c:104-133 — byte-identical stdout. */
void SSS_print_itinfo(const int stop_type, const int iter, const double relres,
                      const double absres, const double factor)
{
    static const char *rule = "-----------------------------------------------------------\n";
    if (iter > 0) {
        printf("%6d | %13.6e   | %13.6e  | %10.4lf\n", iter, relres, absres, factor);
        return;
    }
    fputs(rule, stdout);
    if (stop_type == STOP_REL_RES)
        puts("It Num |   ||r||/||b||   |     ||r||      |  Conv. Factor");
    else if (stop_type == STOP_REL_PRECRES)
        puts("It Num | ||r||_B/||b||_B |    ||r||_B     |  Conv. Factor");
    else if (stop_type == STOP_MOD_REL_RES)
        puts("It Num |   ||r||/||x||   |     ||r||      |  Conv. Factor");
    fputs(rule, stdout);
    printf("%6d | %13.6e   | %13.6e  |     -.-- \n", iter, relres, absres);
}

/* ---- host BLAS-1 (sequential order, as SSS_utils.c:138-260) ------------------------------ */
double SSS_blas_array_norm2(int n, const double *x)
{
    double acc = 0.0;
    for (int i = 0; i < n; ++i) acc += x[i] * x[i];
    return sqrt(acc);
}

double SSS_blas_vec_norm2(const SSS_VEC *x)
{
    return SSS_blas_array_norm2(x->n, x->d);
}

double SSS_blas_array_dot(int n, const double *x, const double *y)
{
    double acc = 0.0;
    for (int i = 0; i < n; ++i) acc += x[i] * y[i];
    return acc;
}

void SSS_blas_array_axpy(int n, double a, const double *x, double *y)
{
    for (int i = 0; i < n; ++i) y[i] += a * x[i];
}

double SSS_blas_array_norminf(int n, const double *x)
{
    double m = 0.0;
    for (int i = 0; i < n; ++i) {
        double v = SSS_ABS(x[i]);
        m = SSS_max(m, v);
    }
    return m;
}

void SSS_blas_array_set(int n, double *x, double Ax)
{
    for (int i = 0; i < n; ++i) x[i] = Ax;
}

void SSS_blas_array_axpby(int n, double a, const double *x, double b, double *y)
{
    for (int i = 0; i < n; ++i) y[i] = a * x[i] + b * y[i];
}

void SSS_blas_array_ax(int n, double a, double *x)
{
    for (int i = 0; i < n; ++i) x[i] *= a;
}

/* ---- allocation and copies (SSS_matvec.c) ------------------------------------------------ */
void sss_huge_hint(void *p, size_t bytes)
{
    if (!p || bytes < ((size_t)8 << 20) || getenv("SSS_NO_HUGEPAGE")) return;
    const uintptr_t pg = 4096, a = ((uintptr_t)p + pg - 1) & ~(pg - 1), e = ((uintptr_t)p + bytes) & ~(pg - 1);
    if (e > a) (void)madvise((void *)a, e - a, MADV_HUGEPAGE);
}

void *sss_big_malloc(size_t bytes)
{
    void *p = malloc(bytes);
    sss_huge_hint(p, bytes);
    return p;
}

void *sss_big_calloc(size_t n, size_t size)
{
    void *p = calloc(n, size);
    sss_huge_hint(p, n * size);
    return p;
}

void *SSS_calloc(size_t size, int type)
{
    size_t bytes = size * (size_t)type;
    void *mem = bytes > 0 ? calloc(size, (size_t)type) : NULL;
    if (mem == NULL) printf("### WARNING: Cannot allocate %.3lf MB RAM!\n", (double)bytes / 1048576);
    sss_huge_hint(mem, bytes);
    return mem;
}

void *SSS_realloc(void *oldmem, size_t tsize)
{
    void *mem = tsize > 0 ? realloc(oldmem, tsize) : NULL;
    if (mem == NULL) printf("### WARNING: Cannot allocate %.3lfMB RAM!\n", (double)tsize / 1048576);
    sss_huge_hint(mem, tsize);
    return mem;
}

SSS_VEC SSS_vec_create(int m)
{
    SSS_VEC v;
    v.n = m;
    v.d = (double *)SSS_calloc((size_t)m, sizeof(double));
    return v;
}

SSS_IVEC SSS_ivec_create(int m)
{
    SSS_IVEC v;
    v.n = m;
    v.d = (int *)SSS_calloc((size_t)m, sizeof(int));
    return v;
}

void SSS_vec_set_value(SSS_VEC *x, double val)
{
    SSS_blas_array_set(x->n, x->d, val);
}

void SSS_vec_destroy(SSS_VEC *u)
{
    if (!u) return;
    free(u->d);
    u->d = NULL;
    u->n = 0;
}

void SSS_ivec_destroy(SSS_IVEC *u)
{
    if (!u) return;
    free(u->d);
    u->d = NULL;
    u->n = 0;
}

void SSS_mat_destroy(SSS_MAT *A)
{
    if (!A) return;
    free(A->row_ptr);
    free(A->col_idx);
    free(A->val);
    A->row_ptr = NULL;
    A->col_idx = NULL;
    A->val = NULL;
}

void SSS_imat_destroy(SSS_IMAT *A)
{
    if (!A) return;
    free(A->row_ptr);
    free(A->col_idx);
    free(A->val);
    A->row_ptr = NULL;
    A->col_idx = NULL;
    A->val = NULL;
}

SSS_MAT SSS_mat_struct_create(int m, int n, int nnz)
{
    SSS_MAT A;
    A.num_rows = m;
    A.num_cols = n;
    A.num_nnzs = nnz;
    A.row_ptr = (int *)SSS_calloc((size_t)m + 1, sizeof(int));
    A.col_idx = nnz > 0 ? (int *)SSS_calloc((size_t)nnz, sizeof(int)) : NULL;
    A.val = nnz > 0 ? (double *)SSS_calloc((size_t)nnz, sizeof(double)) : NULL;
    return A;
}

void SSS_iarray_cp(const int n, int *x, int *y)
{
    memcpy(y, x, (size_t)n * sizeof(int));
}

void SSS_blas_array_cp(int n, const double *x, double *y)
{
    memcpy(y, x, (size_t)n * sizeof(double));
}

void SSS_vec_cp(const SSS_VEC *x, SSS_VEC *y)
{
    y->n = x->n;
    memcpy(y->d, x->d, (size_t)x->n * sizeof(double));
}

void SSS_iarray_set(const int n, int *x, const int Ax)
{
    if (Ax == 0) {
        memset(x, 0, (size_t)n * sizeof(int));
        return;
    }
    for (int i = 0; i < n; ++i) x[i] = Ax;
}

void SSS_mat_cp(SSS_MAT *src, SSS_MAT *des)
{
    des->num_rows = src->num_rows;
    des->num_cols = src->num_cols;
    des->num_nnzs = src->num_nnzs;
    memcpy(des->row_ptr, src->row_ptr, ((size_t)src->num_rows + 1) * sizeof(int));
    memcpy(des->col_idx, src->col_idx, (size_t)src->num_nnzs * sizeof(int));
    memcpy(des->val, src->val, (size_t)src->num_nnzs * sizeof(double));
}

/* SSS_matvec.c:162-187: first diagonal entry of each of the first n rows (0 if absent). */
SSS_VEC SSS_mat_get_diag(SSS_MAT *A, int n)
{
    SSS_VEC diag;
    if (n == 0 || n > A->num_rows || n > A->num_cols) n = SSS_MIN(A->num_rows, A->num_cols);
    diag.n = n;
    diag.d = (double *)SSS_calloc((size_t)n, sizeof(double));
    for (int i = 0; i < n; ++i) {
        for (int k = A->row_ptr[i]; k < A->row_ptr[i + 1]; ++k) {
            if (A->col_idx[k] == i) {
                diag.d[i] = A->val[k];
                break;
            }
        }
    }
    return diag;
}

SSS_AMG SSS_amg_data_create(SSS_AMG_PARS *pars)
{
    SSS_AMG mg;
    memset(&mg, 0, sizeof(mg));
    mg.cg = (SSS_AMG_COMP *)SSS_calloc((size_t)pars->max_levels, sizeof(SSS_AMG_COMP));
    mg.pars = *pars;
    return mg;
}

/* SSS_matvec.c:202-228.  Level-0 b and x belong to the caller and are not freed.  The HBM
 * mirror created by SSS_amg_solve (keyed by mg->cg) is released first. */
void SSS_amg_data_destroy(SSS_AMG *mg)
{
    int nl;
    if (!mg) return;
    sss_dev_release_mirror(mg->cg);
    nl = SSS_max(1, mg->num_levels);
    for (int l = 0; l < nl; ++l) {
        SSS_mat_destroy(&mg->cg[l].A);
        SSS_mat_destroy(&mg->cg[l].P);
        SSS_mat_destroy(&mg->cg[l].R);
        if (l > 0) {
            SSS_vec_destroy(&mg->cg[l].b);
            SSS_vec_destroy(&mg->cg[l].x);
        }
        SSS_vec_destroy(&mg->cg[l].wp);
        SSS_ivec_destroy(&mg->cg[l].cfmark);
    }
    free(mg->cg);
    memset(mg, 0, sizeof(*mg));
}

/*
 * Counting-sort transpose shared by the double and int variants (SSS_matvec.c:247-387).
 * Entries of row j of A^T appear in increasing source-row order, so R = P^T has
 * column-sorted rows — the property the restriction kernel's summation order relies on.
 * The reference's two-slot shifted prefix trick is an implementation detail; what matters is
 * the resulting order, which this reproduces.
 */
static int cmp_int(const void *a, const void *b)
{
    const int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

/* The same transpose with OpenMP: entries are scattered by atomic slot claims, then each output
 * row is sorted by source position -- ascending source row, and stored order inside a row -- which
 * is exactly the order of the sequential fill below, so the result is identical. */
static void transpose_pattern_par(int nrows, int ncols, int nnz, const int *ia, const int *ja,
                                  const void *val, size_t vsize, int *tia, int *tja, void *tval)
{
    int *fill = (int *)sss_big_calloc((size_t)ncols + 1, sizeof(int));
    int *src = (int *)sss_big_malloc(sizeof(int) * (size_t)nnz);
    int *rowof = (int *)sss_big_malloc(sizeof(int) * (size_t)nnz);
    memset(tia, 0, ((size_t)ncols + 1) * sizeof(int));
#pragma omp parallel for schedule(static)
    for (int i = 0; i < nrows; ++i)
        for (int k = ia[i]; k < ia[i + 1]; ++k) {
            rowof[k] = i;
#pragma omp atomic
            tia[ja[k] + 1]++;
        }
    for (int c = 0; c < ncols; ++c) tia[c + 1] += tia[c];
    memcpy(fill, tia, (size_t)ncols * sizeof(int));
#pragma omp parallel for schedule(static)
    for (int k = 0; k < nnz; ++k) {
        int dst;
#pragma omp atomic capture
        dst = fill[ja[k]]++;
        src[dst] = k;
    }
#pragma omp parallel for schedule(dynamic, 4096)
    for (int c = 0; c < ncols; ++c) {
        int *a = src + tia[c];
        const int m = tia[c + 1] - tia[c];
        if (m > 32) {
            qsort(a, (size_t)m, sizeof(int), cmp_int);
        } else {
            for (int t = 1; t < m; ++t) {
                const int key = a[t];
                int u = t - 1;
                while (u >= 0 && a[u] > key) a[u + 1] = a[u], --u;
                a[u + 1] = key;
            }
        }
        for (int t = tia[c]; t < tia[c + 1]; ++t) {
            const int k = src[t];
            tja[t] = rowof[k];
            if (val) memcpy((char *)tval + (size_t)t * vsize, (const char *)val + (size_t)k * vsize, vsize);
        }
    }
    free(src);
    free(rowof);
    free(fill);
}

/* The same transpose without atomics or sorts, for matrices whose rows of one contiguous chunk
 * touch a narrow column window (banded and grid-ordered operators, every AMG level of the stencil
 * workloads): each thread counts its row chunk's entries per column of its own window, the counts
 * of the chunks become per-chunk offsets inside each output row (chunk order = source-row order),
 * and each thread then scatters its rows in stored order -- the sequential fill's order exactly.
 * Returns 0 (nothing written) when the windows together exceed both 4 * ncols and 2^26 ints. */
static int transpose_pattern_chunked(int nrows, int ncols, int nnz, const int *ia, const int *ja,
                                     const void *val, size_t vsize, int *tia, int *tja, void *tval)
{
    const int T = omp_get_max_threads() < 64 ? omp_get_max_threads() : 64;
    int r0[65], lo[64], hi[64];
    int *cnt[64];
    r0[0] = 0;
    for (int t = 1; t < T; ++t) {   /* row chunks of about nnz / T entries */
        const long long want = (long long)nnz * t / T;
        int a = r0[t - 1], b = nrows;
        while (a < b) {
            const int m = a + (b - a) / 2;
            if (ia[m] < want) a = m + 1; else b = m;
        }
        r0[t] = a;
    }
    r0[T] = nrows;
#pragma omp parallel for schedule(static, 1) num_threads(T)
    for (int t = 0; t < T; ++t) {
        int mn = ncols, mx = -1;
        for (int k = ia[r0[t]]; k < ia[r0[t + 1]]; ++k) {
            mn = ja[k] < mn ? ja[k] : mn;
            mx = ja[k] > mx ? ja[k] : mx;
        }
        lo[t] = mn;
        hi[t] = mx;
    }
    long long total = 0;
    for (int t = 0; t < T; ++t) total += hi[t] >= lo[t] ? (long long)(hi[t] - lo[t] + 1) : 0;
    /* SSS_TRANSPOSE_CHUNK_CAP (tests): a lower cap on the windows, so the fallback stays exercised */
    const char *cap_env = getenv("SSS_TRANSPOSE_CHUNK_CAP");
    const long long cap = cap_env ? atoll(cap_env) : 1LL << 26;
    if (total > 4LL * ncols + 4096 && total > cap) return 0;
    int failed = 0;
#pragma omp parallel for schedule(static, 1) num_threads(T) reduction(| : failed)
    for (int t = 0; t < T; ++t) {
        cnt[t] = (int *)sss_big_calloc(hi[t] >= lo[t] ? (size_t)(hi[t] - lo[t] + 1) : 1, sizeof(int));
        if (!cnt[t]) {
            failed = 1;
            continue;
        }
        int *c = cnt[t] - lo[t];
        for (int k = ia[r0[t]]; k < ia[r0[t + 1]]; ++k) c[ja[k]]++;
    }
    if (failed) {   /* out of memory for the windows: nothing written, the atomic transpose runs */
        for (int t = 0; t < T; ++t) free(cnt[t]);
        return 0;
    }
    /* per column: counts -> exclusive offsets of the chunks inside the output row, row length */
    tia[0] = 0;
#pragma omp parallel for schedule(static)
    for (int col = 0; col < ncols; ++col) {
        int run = 0;
        for (int t = 0; t < T; ++t)
            if (col >= lo[t] && col <= hi[t]) {
                int *c = &cnt[t][col - lo[t]];
                const int m = *c;
                *c = run;
                run += m;
            }
        tia[col + 1] = run;
    }
    for (int col = 0; col < ncols; ++col) tia[col + 1] += tia[col];
#pragma omp parallel for schedule(static, 1) num_threads(T)
    for (int t = 0; t < T; ++t) {
        int *c = cnt[t] - lo[t];
        for (int i = r0[t]; i < r0[t + 1]; ++i)
            for (int k = ia[i]; k < ia[i + 1]; ++k) {
                const int dst = tia[ja[k]] + c[ja[k]]++;
                tja[dst] = i;
                if (val) memcpy((char *)tval + (size_t)dst * vsize, (const char *)val + (size_t)k * vsize, vsize);
            }
        free(cnt[t]);
    }
    return 1;
}

static void transpose_pattern(int nrows, int ncols, int nnz, const int *ia, const int *ja,
                              const void *val, size_t vsize, int *tia, int *tja, void *tval)
{
    if (nnz >= (1 << 20)) {
        if (getenv("SSS_TRANSPOSE_ATOMIC") == NULL &&
            transpose_pattern_chunked(nrows, ncols, nnz, ia, ja, val, vsize, tia, tja, tval))
            return;
        transpose_pattern_par(nrows, ncols, nnz, ia, ja, val, vsize, tia, tja, tval);
        return;
    }
    int *fill = (int *)sss_big_calloc((size_t)ncols + 1, sizeof(int));
    memset(tia, 0, ((size_t)ncols + 1) * sizeof(int));
    for (int i = 0; i < nrows; ++i)
        for (int k = ia[i]; k < ia[i + 1]; ++k) tia[ja[k] + 1]++;
    for (int c = 0; c < ncols; ++c) tia[c + 1] += tia[c];
    memcpy(fill, tia, (size_t)ncols * sizeof(int));
    for (int i = 0; i < nrows; ++i) {
        for (int k = ia[i]; k < ia[i + 1]; ++k) {
            int dst = fill[ja[k]]++;
            tja[dst] = i;
            if (val) memcpy((char *)tval + (size_t)dst * vsize, (const char *)val + (size_t)k * vsize, vsize);
        }
    }
    free(fill);
}

SSS_MAT SSS_mat_trans(SSS_MAT *A)
{
    SSS_MAT T;
    T.num_rows = A->num_cols;
    T.num_cols = A->num_rows;
    T.num_nnzs = A->num_nnzs;
    T.row_ptr = (int *)SSS_calloc((size_t)T.num_rows + 1, sizeof(int));
    T.col_idx = (int *)SSS_calloc((size_t)T.num_nnzs, sizeof(int));
    T.val = A->val ? (double *)SSS_calloc((size_t)T.num_nnzs, sizeof(double)) : NULL;
    transpose_pattern(A->num_rows, A->num_cols, A->num_nnzs, A->row_ptr, A->col_idx, A->val,
                      sizeof(double), T.row_ptr, T.col_idx, T.val);
    return T;
}

SSS_IMAT SSS_imat_trans(SSS_IMAT *A)
{
    SSS_IMAT T;
    T.num_rows = A->num_cols;
    T.num_cols = A->num_rows;
    T.num_nnzs = A->num_nnzs;
    T.row_ptr = (int *)SSS_calloc((size_t)T.num_rows + 1, sizeof(int));
    T.col_idx = (int *)SSS_calloc((size_t)T.num_nnzs, sizeof(int));
    T.val = A->val ? (int *)SSS_calloc((size_t)T.num_nnzs, sizeof(int)) : NULL;
    transpose_pattern(A->num_rows, A->num_cols, A->num_nnzs, A->row_ptr, A->col_idx, A->val,
                      sizeof(int), T.row_ptr, T.col_idx, T.val);
    return T;
}

/* ---- roctx ranges (tracing row) --------------------------------------------- */
void sss_trace_push(const char *fmt, ...)
{
    char buf[128];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    roctxRangePushA(buf);
}

void sss_trace_pop(void) { roctxRangePop(); }
