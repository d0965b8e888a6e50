/*
 * sss_mmio.c — Matrix Market ingest and the CLI-side helpers of SSS_main.c.
 *
 * Produces exactly the CSR that the reference's mmio_info/mmio_data build
 * (mmio_highlevel.h:10-305 with mm_read_banner / mm_read_mtx_crd_size, mmio.h:254-367):
 *   - banner tokens are case-insensitive; "symmetric" and "hermitian" mirror every
 *     off-diagonal entry into the transposed row (hermitian without conjugation, as the
 *     reference); "skew-symmetric" and "general" keep only the stored entries;
 *   - within a row, entries keep file order; a mirrored entry lands at its file position;
 *   - pattern -> 1.0, integer -> (double), complex -> real part; duplicates are kept.
 * Numbers are parsed with strtol/strtod (glibc's correctly rounded conversion, identical to
 * fscanf's %d / %lg).
 */
#include "sss_internal.h"

#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

typedef struct {
    int nrows, ncols, nentries;
    char field;     /* 'R' real, 'C' complex, 'I' integer, 'P' pattern */
    int mirrored;   /* symmetric or hermitian */
    int *ri, *ci;   /* 0-based coordinates in file order */
    double *v;
} mtx_triplets;

static void lower(char *s)
{
    for (; *s; ++s) *s = (char)tolower((unsigned char)*s);
}

/* One entry starting at p (the same strtol/strtod sequence as the sequential loop below). */
static const char *parse_entry(const char *p, char field, int *r, int *c, double *v)
{
    char *e;
    long rr = strtol(p, &e, 10), cc;
    double val = 1.0;
    p = e;
    cc = strtol(p, &e, 10);
    p = e;
    if (field == 'R' || field == 'C') {
        val = strtod(p, &e);
        p = e;
        if (field == 'C') { (void)strtod(p, &e); p = e; }
    } else if (field == 'I') {
        val = (double)(int)strtol(p, &e, 10);
        p = e;
    }
    *r = (int)rr - 1;
    *c = (int)cc - 1;
    *v = val;
    return p;
}

/* Large files: the data section is cut into chunks at line ends; each thread counts the entry
 * lines of its chunk, a prefix sum gives every chunk its first entry index, and the chunks are
 * parsed in parallel into their slots -- the same triplets in file order as the sequential loop.
 * Returns 0 (nothing written) when the layout is not one entry per non-blank line with exactly
 * nentries entries, so the sequential parser handles every other case. */
static int parse_parallel(const char *buf, size_t len, mtx_triplets *t)
{
#ifdef _OPENMP
    if (len < ((size_t)4 << 20) || t->nentries <= 0) return 0;
    const int nch = 256;
    size_t cut[257];
    long long cnt[257];
    int ok = 1;
    cut[0] = 0;
    for (int c = 1; c < nch; ++c) {
        size_t q = len / nch * (size_t)c;
        if (q < cut[c - 1]) q = cut[c - 1];
        while (q < len && buf[q] != '\n') ++q;
        cut[c] = q < len ? q + 1 : len;
    }
    cut[nch] = len;
#pragma omp parallel for schedule(dynamic, 1) reduction(&& : ok)
    for (int c = 0; c < nch; ++c) {
        long long n = 0;
        int blank = 1;
        for (size_t q = cut[c]; q < cut[c + 1]; ++q) {
            const char ch = buf[q];
            if (ch == '\n') {
                n += !blank;
                blank = 1;
            } else if (!isspace((unsigned char)ch)) {
                if (blank && ch == '%') ok = 0;   /* comment in the data section */
                blank = 0;
            }
        }
        if (!blank) ++n;
        cnt[c + 1] = n;
    }
    if (!ok) return 0;
    cnt[0] = 0;
    for (int c = 0; c < nch; ++c) cnt[c + 1] += cnt[c];
    if (cnt[nch] != t->nentries) return 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(&& : ok)
    for (int c = 0; c < nch; ++c) {
        const char *p = buf + cut[c], *lim = buf + cut[c + 1];
        for (long long k = cnt[c]; k < cnt[c + 1]; ++k) {
            const char *q = parse_entry(p, t->field, &t->ri[k], &t->ci[k], &t->v[k]);
            if (q > lim || q == p) ok = 0;
            p = q;
            while (p < lim && *p != '\n') {   /* one entry per line: only blanks may follow */
                if (!isspace((unsigned char)*p)) ok = 0;
                ++p;
            }
        }
    }
    return ok;
#else
    (void)buf, (void)len, (void)t;
    return 0;
#endif
}

/* Reads the whole file, returns 0 on success (codes follow mmio_info: -1 open, -2 banner, -4 size). */
static int read_triplets(const char *path, mtx_triplets *t)
{
    FILE *f = fopen(path, "rb");
    char line[1025], banner[64], mtx[64], crd[64], dtype[64], storage[64];
    long pos, end;
    char *buf, *p, *e;

    memset(t, 0, sizeof(*t));
    if (!f) return -1;
    if (!fgets(line, sizeof(line), f) ||
        sscanf(line, "%63s %63s %63s %63s %63s", banner, mtx, crd, dtype, storage) != 5) {
        fclose(f);
        return -2;
    }
    lower(mtx);
    lower(crd);
    lower(dtype);
    lower(storage);
    if (strncmp(banner, "%%MatrixMarket", 14) != 0 || strcmp(mtx, "matrix") != 0 ||
        (strcmp(crd, "coordinate") != 0 && strcmp(crd, "array") != 0)) {
        fclose(f);
        return -2;
    }
    if (!strcmp(dtype, "real")) t->field = 'R';
    else if (!strcmp(dtype, "complex")) t->field = 'C';
    else if (!strcmp(dtype, "pattern")) t->field = 'P';
    else if (!strcmp(dtype, "integer")) t->field = 'I';
    else { fclose(f); return -2; }
    if (!strcmp(storage, "symmetric") || !strcmp(storage, "hermitian")) t->mirrored = 1;
    else if (strcmp(storage, "general") != 0 && strcmp(storage, "skew-symmetric") != 0) {
        fclose(f);
        return -2;
    }
    do {
        if (!fgets(line, sizeof(line), f)) { fclose(f); return -4; }
    } while (line[0] == '%');
    if (sscanf(line, "%d %d %d", &t->nrows, &t->ncols, &t->nentries) != 3) {
        int got;
        do {
            got = fscanf(f, "%d %d %d", &t->nrows, &t->ncols, &t->nentries);
            if (got == EOF) { fclose(f); return -4; }
        } while (got != 3);
    }
    pos = ftell(f);
    fseek(f, 0, SEEK_END);
    end = ftell(f);
    fseek(f, pos, SEEK_SET);
    buf = (char *)sss_big_malloc((size_t)(end - pos) + 1);
    if (fread(buf, 1, (size_t)(end - pos), f) != (size_t)(end - pos)) { /* short read: parse what we got */ }
    buf[end - pos] = '\0';
    fclose(f);

    t->ri = (int *)sss_big_malloc(sizeof(int) * (size_t)(t->nentries > 0 ? t->nentries : 1));
    t->ci = (int *)sss_big_malloc(sizeof(int) * (size_t)(t->nentries > 0 ? t->nentries : 1));
    t->v = (double *)sss_big_malloc(sizeof(double) * (size_t)(t->nentries > 0 ? t->nentries : 1));
    if (parse_parallel(buf, (size_t)(end - pos), t)) {
        free(buf);
        return 0;
    }
    p = buf;
    for (int k = 0; k < t->nentries; ++k) {
        long r = strtol(p, &e, 10);
        long c;
        double val = 1.0;
        p = e;
        c = strtol(p, &e, 10);
        p = e;
        if (t->field == 'R' || t->field == 'C') {
            val = strtod(p, &e);
            p = e;
            if (t->field == 'C') { (void)strtod(p, &e); p = e; }
        } else if (t->field == 'I') {
            val = (double)(int)strtol(p, &e, 10);
            p = e;
        }
        t->ri[k] = (int)r - 1;
        t->ci[k] = (int)c - 1;
        t->v[k] = val;
    }
    free(buf);
    return 0;
}

static void free_triplets(mtx_triplets *t)
{
    free(t->ri);
    free(t->ci);
    free(t->v);
}

/* Row counts including mirrored off-diagonals; fills rp[0..nrows] as an exclusive scan. */
static int build_row_ptr(const mtx_triplets *t, int *rp)
{
    memset(rp, 0, sizeof(int) * ((size_t)t->nrows + 1));
    for (int k = 0; k < t->nentries; ++k) {
        rp[t->ri[k] + 1]++;
        if (t->mirrored && t->ri[k] != t->ci[k]) rp[t->ci[k] + 1]++;
    }
    for (int i = 0; i < t->nrows; ++i) rp[i + 1] += rp[i];
    return rp[t->nrows];
}

/* mmio_info parses the file and SSS_mat_read then calls mmio_data on the same file: the triplets
 * of the last mmio_info are kept for it (keyed by path, size and modification time), so a matrix
 * is parsed once. */
static struct {
    char path[4096];
    off_t size;
    struct timespec mtime;
    int valid;
    mtx_triplets t;
} last_parse;

static int file_key(const char *path, off_t *size, struct timespec *mtime)
{
    struct stat st;
    if (stat(path, &st) != 0) return 0;
    *size = st.st_size;
    *mtime = st.st_mtim;
    return 1;
}

static void drop_last_parse(void)
{
    if (last_parse.valid) free_triplets(&last_parse.t);
    last_parse.valid = 0;
}

int mmio_info(int *m, int *n, int *nnz, int *isSymmetric, char *filename)
{
    mtx_triplets t;
    int rc = read_triplets(filename, &t);
    int *rp;
    if (rc != 0) return rc;
    rp = (int *)sss_big_malloc(sizeof(int) * ((size_t)t.nrows + 1));
    *m = t.nrows;
    *n = t.ncols;
    *nnz = build_row_ptr(&t, rp);
    *isSymmetric = t.mirrored;
    free(rp);
    drop_last_parse();
    if (strlen(filename) < sizeof(last_parse.path) && file_key(filename, &last_parse.size, &last_parse.mtime)) {
        strcpy(last_parse.path, filename);
        last_parse.t = t;
        last_parse.valid = 1;
    } else {
        free_triplets(&t);
    }
    return 0;
}

int mmio_data(int *csrRowPtr, int *csrColIdx, double *csrAx, char *filename)
{
    mtx_triplets t;
    int rc = 0;
    int *next;
    off_t size;
    struct timespec mt;
    if (last_parse.valid && !strcmp(last_parse.path, filename) && file_key(filename, &size, &mt) &&
        size == last_parse.size && mt.tv_sec == last_parse.mtime.tv_sec && mt.tv_nsec == last_parse.mtime.tv_nsec) {
        t = last_parse.t;
        last_parse.valid = 0;
    } else {
        drop_last_parse();
        rc = read_triplets(filename, &t);
    }
    if (rc != 0) return rc;
    build_row_ptr(&t, csrRowPtr);
    next = (int *)sss_big_malloc(sizeof(int) * ((size_t)t.nrows + 1));
    memcpy(next, csrRowPtr, sizeof(int) * ((size_t)t.nrows + 1));
    for (int k = 0; k < t.nentries; ++k) {
        int r = t.ri[k], c = t.ci[k], dst = next[r]++;
        csrColIdx[dst] = c;
        csrAx[dst] = t.v[k];
        if (t.mirrored && r != c) {
            dst = next[c]++;
            csrColIdx[dst] = r;
            csrAx[dst] = t.v[k];
        }
    }
    free(next);
    free_triplets(&t);
    return 0;
}

/* SSS_main.c:12-22 */
void SSS_mat_read(char *filemat, SSS_MAT *A)
{
    int sym = 0, rc;
    printf("filename: %s\n", filemat);
    rc = mmio_info(&A->num_rows, &A->num_cols, &A->num_nnzs, &sym, filemat);
    if (rc != 0) SSS_exit_on_errcode(rc == -1 ? ERROR_OPEN_FILE : ERROR_WRONG_FILE, __func__);
    A->row_ptr = (int *)sss_big_malloc(((size_t)A->num_rows + 1) * sizeof(int));
    A->col_idx = (int *)sss_big_malloc((size_t)(A->num_nnzs > 0 ? A->num_nnzs : 1) * sizeof(int));
    A->val = (double *)sss_big_malloc((size_t)(A->num_nnzs > 0 ? A->num_nnzs : 1) * sizeof(double));
    mmio_data(A->row_ptr, A->col_idx, A->val, filemat);
    printf("A: m = %d, n = %d, nnz = %d\n", A->num_rows, A->num_cols, A->num_nnzs);
}

/* SSS_main.c:25-64 — the reference defaults. */
void SSS_amg_pars_init(SSS_AMG_PARS *pars)
{
    memset(pars, 0, sizeof(*pars));
    pars->smoother = SSS_SM_GS;
    pars->max_it = 100;
    pars->tol = 1e-6;
    pars->ctol = 1e-7;
    pars->max_levels = 30;
    pars->coarse_dof = MIN_CDOF;
    pars->cycle_type = 1;
    pars->cf_order = 1;
    pars->pre_iter = 2;
    pars->post_iter = 2;
    pars->relax = 1.0;
    pars->poly_deg = 3;
    pars->cs_type = SSS_COARSE_RS;
    pars->interp_type = intERP_DIR;
    pars->max_row_sum = 0.9;
    pars->strong_threshold = 0.3;
    pars->trunc_threshold = 0.2;
}

/* SSS_main.c:67-119 — byte-identical stdout. */
void SSS_amg_pars_print(SSS_AMG_PARS *pars)
{
    static const char *rule = "-----------------------------------------------------------\n";
    printf("\n               AMG Parameters \n");
    fputs(rule, stdout);
    printf("AMG max num of iter:               %d\n", pars->max_it);
    printf("AMG tol:                           %g\n", pars->tol);
    printf("AMG ctol:                          %g\n", pars->ctol);
    printf("AMG max levels:                    %d\n", pars->max_levels);
    printf("AMG cycle type:                    %d\n", pars->cycle_type);
    printf("AMG smoother type:                 %d\n", pars->smoother);
    printf("AMG smoother order:                %d\n", pars->cf_order);
    printf("AMG num of presmoothing:           %d\n", pars->pre_iter);
    printf("AMG num of postsmoothing:          %d\n", pars->post_iter);
    if (pars->smoother == SSS_SM_SOR || pars->smoother == SSS_SM_SSOR ||
        pars->smoother == SSS_SM_GSOR || pars->smoother == SSS_SM_SGSOR)
        printf("AMG relax factor:                  %.4lf\n", pars->relax);
    else if (pars->smoother == SSS_SM_POLY)
        printf("AMG polynomial smoother degree:    %d\n", pars->poly_deg);
    printf("AMG coarsening type:               %d\n", pars->cs_type);
    if (pars->interp_type == intERP_DIR)
        printf("AMG interPolation type:            Dir\n");
    else if (pars->interp_type == intERP_STD)
        printf("AMG interPolation type:            STD\n");
    printf("AMG dof on coarsest grid:          %d\n", pars->coarse_dof);
    printf("AMG strong threshold:              %.4lf\n", pars->strong_threshold);
    printf("AMG truncation threshold:          %.4lf\n", pars->trunc_threshold);
    printf("AMG max row sum:                   %.4lf\n", pars->max_row_sum);
    fputs(rule, stdout);
}
