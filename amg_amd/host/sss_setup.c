/*
 * sss_setup.c — AMG setup phase (host C).  Out of the GPU hot-path scope (SURVEY.md §2 rows
 * 10-12), but it builds the hierarchy the hot path consumes, so it reproduces the reference's
 * setup semantics exactly ("uncapped" reference):
 *
 *   strong couplings ............ Setup/SSS_coarsen.c:106-181
 *   weak-coupling compression ... Setup/SSS_coarsen.c:185-212
 *   classical RS C/F split ...... Setup/SSS_coarsen.c:294-498 (bucketed measure lists)
 *   F-F cleanup ................. Setup/SSS_coarsen.c:501-574
 *   direct P pattern ............ Setup/SSS_coarsen.c:577-630
 *   direct interpolation ........ Setup/SSS_inter.cu:400-547 (the host twin interp_DIR)
 *   standard P pattern .......... Setup/SSS_coarsen.c:633-725 (interp_type 2)
 *   standard interpolation ...... Setup/SSS_inter.cu:550-715 (interp_STD)
 *   truncation .................. Setup/SSS_inter.cu:16-102
 *   Galerkin RAP ................ SSS_matvec.c:398-534
 *   level loop .................. Setup/SSS_SETUP.cu:36-178
 *
 * The measure lists are kept as an array of FIFO buckets indexed by measure instead of the
 * reference's heap-allocated sorted list of list nodes with element-level linked lists
 * (lists/where); every insert/remove happens in the same order, so the head of the maximal
 * bucket — the next C point — is the same.  RAP runs the reference's row-by-row
 * marker algorithm independently per coarse row (OpenMP), which yields identical rows
 * (diagonal first, then discovery order; identical summation order).
 */
#include "sss_internal.h"

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <unistd.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ======================================================================================
 * Strength of connection
 * ====================================================================================== */
static void strong_couplings(const SSS_MAT *A, SSS_IMAT *S, const SSS_AMG_PARS *pars)
{
    const int n = A->num_rows;
    const double theta = pars->strong_threshold;
    const double row_sum_bound = 2.0 - pars->max_row_sum;
    const int *ia = A->row_ptr, *ja = A->col_idx;
    const double *a = A->val;

    S->num_rows = n;
    S->num_cols = A->num_cols;
    S->num_nnzs = A->num_nnzs;
    S->val = NULL;
    S->row_ptr = (int *)SSS_calloc((size_t)n + 1, sizeof(int));
    S->col_idx = (int *)SSS_calloc((size_t)A->num_nnzs, sizeof(int));
    memcpy(S->row_ptr, ia, ((size_t)n + 1) * sizeof(int));
    memcpy(S->col_idx, ja, (size_t)A->num_nnzs * sizeof(int));

#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        double abs_sum = 0.0, max_off = 0.0, dii = 0.0;
        int have_diag = 0;
        for (int k = ia[i]; k < ia[i + 1]; ++k) {
            double m = SSS_ABS(a[k]);
            abs_sum += m;
            if (ja[k] != i) max_off = SSS_max(max_off, m);
            else if (!have_diag) { dii = a[k]; have_diag = 1; }
        }
        max_off *= theta;
        for (int k = ia[i]; k < ia[i + 1]; ++k)     /* first diagonal entry is never strong */
            if (ja[k] == i) { S->col_idx[k] = -1; break; }
        if (abs_sum < row_sum_bound * SSS_ABS(dii)) {
            for (int k = ia[i]; k < ia[i + 1]; ++k) S->col_idx[k] = -1;
        } else {
            for (int k = ia[i]; k < ia[i + 1]; ++k)
                if (-a[k] <= max_off) S->col_idx[k] = -1;
        }
    }
}

/* Drops entries marked -1; returns -99 when nothing strong is left (reference's ERROR_UNKNOWN). */
static int drop_weak(SSS_IMAT *S)
{
    const int n = S->num_rows;
    if (S->num_nnzs < (1 << 20)) {
        int out = 0;
        for (int i = 0; i < n; ++i) {
            int lo = S->row_ptr[i], hi = S->row_ptr[i + 1];
            S->row_ptr[i] = out;
            for (int k = lo; k < hi; ++k)
                if (S->col_idx[k] > -1) S->col_idx[out++] = S->col_idx[k];
        }
        S->row_ptr[n] = out;
        S->num_nnzs = out;
        return out > 0 ? 0 : -99;
    }
    /* same compaction in parallel: kept counts per row, prefix sum, copy into a new array */
    int *cnt = (int *)SSS_calloc((size_t)n + 1, sizeof(int));
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        int c = 0;
        for (int k = S->row_ptr[i]; k < S->row_ptr[i + 1]; ++k) c += S->col_idx[k] > -1;
        cnt[i + 1] = c;
    }
    for (int i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
    const int out = cnt[n];
    int *ci = (int *)SSS_calloc((size_t)(out > 0 ? out : 1), sizeof(int));
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        int o = cnt[i];
        for (int k = S->row_ptr[i]; k < S->row_ptr[i + 1]; ++k)
            if (S->col_idx[k] > -1) ci[o++] = S->col_idx[k];
    }
    free(S->col_idx);
    free(S->row_ptr);
    S->col_idx = ci;
    S->row_ptr = cnt;
    S->num_nnzs = out;
    return out > 0 ? 0 : -99;
}

/* ======================================================================================
 * Measure buckets.  The reference keeps one doubly linked list per measure (SSS_coarsen.c
 * lists/where + list nodes): inserts append at the tail, the next C point is the head of the
 * largest non-empty list -- i.e. among the points of maximal measure, the one inserted
 * earliest.  Here each bucket is an append-only FIFO array of (point, version) entries and a
 * removal only bumps the point's version (its entry goes stale and is skipped when it reaches
 * the head).  Same head, same order of picks, but a move is two sequential writes instead of
 * four dependent pointer updates scattered over the grid (the serial first pass is
 * memory-latency bound).  Buckets are compacted in place (order kept) when most of their
 * entries are stale.
 * ====================================================================================== */
typedef struct {
    int pt;
    unsigned ver;
} bucket_entry;

typedef struct {
    bucket_entry *e;
    size_t head, tail, cap;
    int live;                /* live entries = points in this bucket */
} bucket_fifo;

/* Per-point state of the first pass in one 8-byte record (one cache line holds eight points; the
 * pass touches measure, mark and version of the same neighbours).  A point's version moves once
 * per bucket move -- a few dozen times at most -- so 29 bits never wrap. */
typedef struct {
    int lambda;              /* measure */
    int mark : 3;            /* UNPT / CGPT / FGPT / ISPT */
    unsigned ver : 29;       /* current version: a bucket entry is live iff it matches */
} rs_point;

typedef struct {
    bucket_fifo *b;          /* per measure */
    int cap;                 /* allocated measures */
    int top;                 /* upper bound on the largest non-empty measure */
    rs_point *pts;
} measure_buckets;

static void buckets_grow(measure_buckets *B, int m)
{
    int old = B->cap, cap = B->cap;
    while (cap <= m) cap = cap * 2 + 16;
    B->b = (bucket_fifo *)realloc(B->b, sizeof(bucket_fifo) * (size_t)cap);
    memset(B->b + old, 0, sizeof(bucket_fifo) * (size_t)(cap - old));
    B->cap = cap;
}

static void bucket_compact(bucket_fifo *q, const rs_point *pts)
{
    size_t o = 0;
    for (size_t k = q->head; k < q->tail; ++k)
        if (q->e[k].ver == pts[q->e[k].pt].ver) q->e[o++] = q->e[k];
    q->head = 0;
    q->tail = o;
}

static inline void bucket_insert(measure_buckets *B, int m, int pt)
{
    if (m >= B->cap) buckets_grow(B, m);
    bucket_fifo *q = &B->b[m];
    if (q->tail == q->cap) {
        if (q->tail - q->head > 2 * (size_t)q->live + 64 || q->head > q->cap / 2) bucket_compact(q, B->pts);
        if (q->tail == q->cap) {
            q->cap = q->cap * 2 + 256;
            q->e = (bucket_entry *)realloc(q->e, sizeof(bucket_entry) * q->cap);
        }
    }
    q->e[q->tail].pt = pt;
    q->e[q->tail].ver = ++B->pts[pt].ver;
    q->tail++;
    q->live++;
    if (m > B->top) B->top = m;
}

static inline void bucket_remove(measure_buckets *B, int m, int pt)
{
    if (m < 0 || m >= B->cap || B->b[m].live == 0) {
        printf("### ERROR: This list is empty! %s : %d\n", __FILE__, __LINE__);
        return;
    }
    B->pts[pt].ver++;
    if (--B->b[m].live == 0) B->b[m].head = B->b[m].tail = 0;
}

/* bucket_remove(from) + bucket_insert(to) with one version step: the insert's new version already
 * makes the old entry stale (same buckets, same order as the two calls). */
static inline void bucket_move(measure_buckets *B, int from, int to, int pt)
{
    if (from < 0 || from >= B->cap || B->b[from].live == 0) {
        printf("### ERROR: This list is empty! %s : %d\n", __FILE__, __LINE__);
        return;
    }
    if (--B->b[from].live == 0) B->b[from].head = B->b[from].tail = 0;
    bucket_insert(B, to, pt);
}

/* Head point of the largest non-empty bucket, or -1 if every bucket is empty. */
static int bucket_max_head(measure_buckets *B)
{
    while (B->top > 0 && B->b[B->top].live == 0) B->top--;
    if (B->top <= 0) return -1;
    bucket_fifo *q = &B->b[B->top];
    while (q->e[q->head].ver != B->pts[q->e[q->head].pt].ver) q->head++;
    for (size_t t = q->head + 1; t < q->tail && t < q->head + 4; ++t) __builtin_prefetch(&B->pts[q->e[t].pt]);
    return q->e[q->head].pt;
}

/* Rows that can change in the C1 and F-F passes below.  Both passes visit the F rows in order and
 * act only on a row with a strongly coupled F neighbour j that shares no strong C point with it
 * (an "unshared pair").  Between rows, marks only ever move F -> C (a tentative C point that is
 * reverted was F before), so the C set only grows: a row with no unshared pair under the marks
 * before the pass never gets one, and the pass does nothing there but per-row bookkeeping.  This
 * flags the rows that have an unshared pair under the starting marks, row-parallel; the serial
 * passes run their exact logic on the flagged rows only.  owner (n ints) is a scratch marker
 * shared by the threads: a concurrent overwrite can only hide a shared C point, so it can add
 * rows (checked serially anyway), never drop one.  Returns owner reset to -1. */
static char *flag_unshared_rows(const SSS_IMAT *S, const int *mark, int *owner)
{
    const int n = S->num_rows;
    char *flag = (char *)SSS_calloc((size_t)(n > 0 ? n : 1), 1);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) __atomic_store_n(&owner[i], -1, __ATOMIC_RELAXED);
#pragma omp parallel for schedule(dynamic, 4096)
    for (int i = 0; i < n; ++i) {
        if (mark[i] != FGPT) continue;
        for (int q = S->row_ptr[i]; q < S->row_ptr[i + 1]; ++q)
            if (mark[S->col_idx[q]] == CGPT) __atomic_store_n(&owner[S->col_idx[q]], i, __ATOMIC_RELAXED);
        for (int q = S->row_ptr[i]; q < S->row_ptr[i + 1] && !flag[i]; ++q) {
            const int j = S->col_idx[q];
            int shares = 0;
            if (mark[j] != FGPT) continue;
            for (int r = S->row_ptr[j]; r < S->row_ptr[j + 1]; ++r)
                if (__atomic_load_n(&owner[S->col_idx[r]], __ATOMIC_RELAXED) == i) { shares = 1; break; }
            if (!shares) flag[i] = 1;
        }
    }
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) owner[i] = -1;
    return flag;
}

#ifndef PF_DEPTH
#define PF_DEPTH 5
#endif

/* Classical Ruge-Stueben first pass + C1 fix-up.  Returns the C-point count (or <0). */
static int rs_split(const SSS_MAT *A, SSS_IMAT *S, SSS_IVEC *vertices)
{
    const int n = A->num_rows;
    int *mark = vertices->d;
    int ncoarse, undecided = 0;
    int *lambda, *owner;
    SSS_IMAT ST;
    measure_buckets B;

    const int timing = getenv("SSS_SETUP_TIMING") != NULL;
    const double t0 = SSS_get_time();
    ncoarse = drop_weak(S);
    if (ncoarse < 0) return ncoarse;
    const double tdrop = SSS_get_time();
    ST = SSS_imat_trans(S);
    const double t1 = SSS_get_time();

    memset(&B, 0, sizeof(B));
    B.pts = (rs_point *)SSS_calloc((size_t)n, sizeof(rs_point));
    rs_point *P = B.pts;
    buckets_grow(&B, 64);

#pragma omp parallel for schedule(static) reduction(+ : undecided) if (n > 65536)
    for (int i = 0; i < n; ++i) {
        if (S->row_ptr[i + 1] == S->row_ptr[i]) {
            P[i].mark = ISPT;
            P[i].lambda = 0;
        } else {
            P[i].mark = UNPT;
            P[i].lambda = ST.row_ptr[i + 1] - ST.row_ptr[i];
            undecided++;
        }
    }

    /* Initial lists; points with no influence become F immediately. */
    for (int i = 0; i < n; ++i) {
        if (P[i].mark == ISPT) continue;
        if (P[i].lambda > 0) {
            bucket_insert(&B, P[i].lambda, i);
            continue;
        }
        if (P[i].lambda < 0) printf("### WARNING: Negative lambda[%d]!\n", i);
        P[i].mark = FGPT;
        undecided--;
        for (int k = S->row_ptr[i]; k < S->row_ptr[i + 1]; ++k) {
            int j = S->col_idx[k];
            if (P[j].mark == ISPT) continue;
            if (j < i) {
                if (P[j].lambda > 0) bucket_remove(&B, P[j].lambda, j);
                P[j].lambda++;
                bucket_insert(&B, P[j].lambda, j);
            } else {
                P[j].lambda++;
            }
        }
    }

    const double t2 = SSS_get_time();
    while (undecided > 0) {
        int c = bucket_max_head(&B);
        int mc;
        if (c < 0) {
            printf("### ERROR: RS coarsening ran out of candidates (%d undecided)\n", undecided);
            break;
        }
        /* The pass is bound by cache misses on the neighbourhood of each pick (≈35 dependent
         * record / row accesses per pick, spread over three grid planes): request them all up
         * front -- the records of c's neighbours, their S rows, and the records of the S rows of
         * the neighbours that are about to become F. */
        {   /* and, pipelined, the neighbourhoods of the next candidates in the top bucket (the
             * likely next picks): row pointers PF_DEPTH picks ahead, their rows two ahead, the
             * records of their neighbours one ahead -- each stage reads only what an earlier pick
             * has already requested */
            const bucket_fifo *tq = &B.b[B.top];
            const size_t end = tq->tail < tq->head + 1 + PF_DEPTH ? tq->tail : tq->head + 1 + PF_DEPTH;
            for (size_t t = tq->head + 1; t < end; ++t) {
                const int nx = tq->e[t].pt;
                const size_t d = t - tq->head;
                if (d >= 3) {
                    __builtin_prefetch(&ST.row_ptr[nx]);
                    __builtin_prefetch(&S->row_ptr[nx]);
                } else if (d == 2) {
                    __builtin_prefetch(ST.col_idx + ST.row_ptr[nx]);
                    __builtin_prefetch(S->col_idx + S->row_ptr[nx]);
                } else {
                    for (int q = ST.row_ptr[nx]; q < ST.row_ptr[nx + 1]; ++q) __builtin_prefetch(&P[ST.col_idx[q]], 1);
                    for (int q = S->row_ptr[nx]; q < S->row_ptr[nx + 1]; ++q) __builtin_prefetch(&P[S->col_idx[q]], 1);
                }
            }
        }
        for (int q = ST.row_ptr[c]; q < ST.row_ptr[c + 1]; ++q) {
            const int j = ST.col_idx[q];
            __builtin_prefetch(&P[j], 1);
            __builtin_prefetch(&S->row_ptr[j]);
        }
        for (int q = S->row_ptr[c]; q < S->row_ptr[c + 1]; ++q) __builtin_prefetch(&P[S->col_idx[q]], 1);
        for (int q = ST.row_ptr[c]; q < ST.row_ptr[c + 1]; ++q) __builtin_prefetch(S->col_idx + S->row_ptr[ST.col_idx[q]]);
        for (int q = ST.row_ptr[c]; q < ST.row_ptr[c + 1]; ++q) {
            const int j = ST.col_idx[q];
            if (P[j].mark != UNPT) continue;
            for (int r = S->row_ptr[j]; r < S->row_ptr[j + 1]; ++r) __builtin_prefetch(&P[S->col_idx[r]], 1);
        }
        mc = P[c].lambda;
        if (mc == 0) printf("### WARNING: Head of the list has measure 0!\n");
        P[c].mark = CGPT;
        P[c].lambda = 0;
        undecided--;
        bucket_remove(&B, mc, c);
        ncoarse++;

        /* points that c strongly influences become F */
        for (int q = ST.row_ptr[c]; q < ST.row_ptr[c + 1]; ++q) {
            int j = ST.col_idx[q];
            if (P[j].mark != UNPT) continue;
            P[j].mark = FGPT;
            bucket_remove(&B, P[j].lambda, j);
            undecided--;
            for (int r = S->row_ptr[j]; r < S->row_ptr[j + 1]; ++r) {
                int k = S->col_idx[r];
                if (P[k].mark != UNPT) continue;
                bucket_move(&B, P[k].lambda, P[k].lambda + 1, k);
                P[k].lambda++;
            }
        }
        /* points that strongly influence c lose one unit of measure */
        for (int q = S->row_ptr[c]; q < S->row_ptr[c + 1]; ++q) {
            int j = S->col_idx[q], m;
            if (P[j].mark != UNPT) continue;
            m = P[j].lambda;
            if (m - 1 > 0) {
                bucket_move(&B, m, m - 1, j);
                P[j].lambda = m - 1;
                continue;
            }
            bucket_remove(&B, m, j);
            P[j].lambda = --m;
            P[j].mark = FGPT;
            undecided--;
            for (int r = S->row_ptr[j]; r < S->row_ptr[j + 1]; ++r) {
                int k = S->col_idx[r];
                if (P[k].mark != UNPT) continue;
                bucket_move(&B, P[k].lambda, P[k].lambda + 1, k);
                P[k].lambda++;
            }
        }
    }

    const double t3 = SSS_get_time();
    lambda = (int *)SSS_calloc((size_t)n, sizeof(int));
    for (int i = 0; i < n; ++i) mark[i] = P[i].mark;
    free(B.pts);
    /* C1 criterion: two strongly coupled F points must share a strong C point. */
    owner = lambda;
    char *maybe = flag_unshared_rows(S, mark, owner);   /* the rows this pass can change */
    for (int i = 0; i < n; ++i) {
        int promoted = -1, have_promoted = 0;
        if (!maybe[i] || mark[i] != FGPT) continue;
        for (int q = S->row_ptr[i]; q < S->row_ptr[i + 1]; ++q)
            if (mark[S->col_idx[q]] == CGPT) owner[S->col_idx[q]] = i;
        for (int q = S->row_ptr[i]; q < S->row_ptr[i + 1]; ++q) {
            int j = S->col_idx[q], shares = 0;
            if (mark[j] != FGPT) continue;
            for (int r = S->row_ptr[j]; r < S->row_ptr[j + 1]; ++r)
                if (owner[S->col_idx[r]] == i) { shares = 1; break; }
            if (shares) continue;
            if (!have_promoted) {
                mark[j] = CGPT;
                ncoarse++;
                owner[j] = i;
                promoted = j;
                have_promoted = 1;
            } else {
                mark[i] = CGPT;
                mark[promoted] = FGPT;
                break;
            }
        }
    }
    free(maybe);

    if (timing)
        fprintf(stderr, "[setup]   RS split: drop %.3f s, transpose %.3f s, lists %.3f s, first pass %.3f s, C1 %.3f s\n",
                tdrop - t0, t1 - tdrop, t2 - t1, t3 - t2, SSS_get_time() - t3);
    SSS_imat_destroy(&ST);
    for (int m = 0; m < B.cap; ++m) free(B.b[m].e);
    free(B.b);
    free(lambda);
    return ncoarse;
}

/* Setup/SSS_coarsen.c:501-574.  Note: the tentative-C state (pending, pending_owner,
 * tentative) deliberately persists across rows exactly as in the reference. */
static int cleanup_ff(const SSS_IMAT *S, SSS_IVEC *vertices, int n, int ncoarse)
{
    int *mark = vertices->d;
    int *tag = (int *)SSS_calloc((size_t)n, sizeof(int));
    int pending = FALSE, pending_owner = -1, tentative = -1;
    char *maybe = flag_unshared_rows(S, mark, tag);   /* the rows this pass can change; tag = -1 */

    for (int i = 0; i < n; ++i) {
        if (mark[i] != FGPT) continue;
        if (!maybe[i]) {   /* no unshared pair: the row only resets the tentative C point */
            if (pending_owner != i) tentative = -1;
            continue;
        }
        for (int q = S->row_ptr[i]; q < S->row_ptr[i + 1]; ++q) {
            int j = S->col_idx[q];
            tag[j] = (mark[j] == CGPT) ? i : -1;
        }
        if (pending_owner != i) tentative = -1;
        for (int q = S->row_ptr[i]; q < S->row_ptr[i + 1]; ++q) {
            int j = S->col_idx[q], linked = 0;
            if (mark[j] != FGPT) continue;
            for (int r = S->row_ptr[j]; r < S->row_ptr[j + 1]; ++r)
                if (tag[S->col_idx[r]] == i) { linked = 1; break; }
            if (linked) continue;
            if (pending) {
                mark[i] = CGPT;
                ncoarse++;
                if (tentative > -1) {
                    mark[tentative] = FGPT;
                    ncoarse--;
                    tentative = -1;
                }
                pending = FALSE;
            } else {
                mark[j] = CGPT;
                ncoarse++;
                tentative = j;
                pending_owner = i;
                pending = TRUE;
                i--;                    /* revisit i with j as a C point */
            }
            break;
        }
    }
    free(maybe);
    free(tag);
    return ncoarse;
}

/* Setup/SSS_coarsen.c:577-630: F rows take their strong C neighbours, C rows themselves. */
static void direct_pattern(SSS_MAT *P, const SSS_IMAT *S, const SSS_IVEC *vertices, int n, int ncoarse)
{
    const int *mark = vertices->d;
    int pos = 0;
    P->num_rows = n;
    P->num_cols = ncoarse;
    P->row_ptr = (int *)SSS_calloc((size_t)n + 1, sizeof(int));
    /* row counts in parallel, prefix, then each row fills its own span (same arrays as the
     * reference's sequential pass) */
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int i = 0; i < n; ++i) {
        int cnt = 0;
        if (mark[i] == FGPT) {
            for (int q = S->row_ptr[i]; q < S->row_ptr[i + 1]; ++q)
                if (mark[S->col_idx[q]] == CGPT) cnt++;
        } else if (mark[i] == CGPT) {
            cnt = 1;
        }
        P->row_ptr[i + 1] = cnt;
    }
    for (int i = 0; i < n; ++i) P->row_ptr[i + 1] += P->row_ptr[i];
    P->num_nnzs = P->row_ptr[n] - P->row_ptr[0];
    P->col_idx = (int *)SSS_calloc((size_t)P->num_nnzs, sizeof(int));
    P->val = (double *)SSS_calloc((size_t)P->num_nnzs, sizeof(double));
    (void)pos;
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int i = 0; i < n; ++i) {
        int o = P->row_ptr[i];
        if (mark[i] == FGPT) {
            for (int q = S->row_ptr[i]; q < S->row_ptr[i + 1]; ++q)
                if (mark[S->col_idx[q]] == CGPT) P->col_idx[o++] = S->col_idx[q];
        } else if (mark[i] == CGPT) {
            P->col_idx[o] = i;
        }
    }
}

/* Per-thread scratch of a row-parallel loop: one buffer of `bytes` for each of up to
 * omp_get_max_threads() threads (at most 256), all of them together within a quarter of the
 * machine's memory (at least 2 GiB), fewer threads when an allocation fails.  Returns the threads
 * that got one; the loop runs on that many.  With none (even one buffer failed) the setup cannot go
 * on: the reference's allocation failure path (a warning, then the error exit). */
enum { kScratchMax = 256 };
static int scratch_alloc(size_t bytes, void **buf)
{
    const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
    size_t budget = (pages > 0 && psz > 0) ? (size_t)pages * (size_t)psz / 4 : 0;
    if (budget < ((size_t)2 << 30)) budget = (size_t)2 << 30;
    if (bytes == 0) bytes = 1;
    int T = omp_get_max_threads();
    if (T > kScratchMax) T = kScratchMax;
    while (T > 1 && (size_t)T * bytes > budget) T--;
    int got = 0;
    while (got < T && (buf[got] = malloc(bytes)) != NULL) ++got;
    if (got == 0) {
        printf("### WARNING: Cannot allocate %.3lf MB RAM!\n", (double)bytes / 1048576);
        SSS_exit_on_errcode(ERROR_ALLOC_MEM, __func__);
    }
    return got;
}
static void scratch_free(void **buf, int T)
{
    for (int t = 0; t < T; ++t) free(buf[t]);
}

/* Setup/SSS_coarsen.c:633-725 (form_P_pattern_std): an F row takes its strong C neighbours and the
 * strong C neighbours of its strong F neighbours, each once, in discovery order; a C row its own
 * index; any other row nothing.  The reference's one `visited` array only ever answers "taken by
 * this row already?", so rows are independent: two row-parallel passes (count, then fill at the
 * prefix offsets), each thread with its own row-stamped array. */
static void std_pattern(SSS_MAT *P, const SSS_IMAT *S, const SSS_IVEC *vertices, int n, int ncoarse)
{
    const int *mark = vertices->d;
    void *scr[kScratchMax];
    const int T = scratch_alloc(sizeof(int) * (size_t)(n > 0 ? n : 1), scr);
    P->num_rows = n;
    P->num_cols = ncoarse;
    P->row_ptr = (int *)SSS_calloc((size_t)n + 1, sizeof(int));
    for (int fill = 0; fill < 2; ++fill) {
        if (fill) {
            for (int i = 0; i < n; ++i) P->row_ptr[i + 1] += P->row_ptr[i];
            P->num_nnzs = P->row_ptr[n] - P->row_ptr[0];
            P->col_idx = (int *)SSS_calloc((size_t)(P->num_nnzs > 0 ? P->num_nnzs : 1), sizeof(int));
            P->val = (double *)SSS_calloc((size_t)(P->num_nnzs > 0 ? P->num_nnzs : 1), sizeof(double));
        }
#pragma omp parallel num_threads(T) if (n > 4096)
        {
            int *seen = (int *)scr[omp_get_thread_num()];
            for (int i = 0; i < n; ++i) seen[i] = -1;
#pragma omp for schedule(dynamic, 1024)
            for (int i = 0; i < n; ++i) {
                int cnt = 0, o = fill ? P->row_ptr[i] : 0;
                if (mark[i] == FGPT) {
                    for (int q = S->row_ptr[i]; q < S->row_ptr[i + 1]; ++q) {
                        const int k = S->col_idx[q];
                        if (mark[k] == CGPT && seen[k] != i) {
                            seen[k] = i;
                            if (fill) P->col_idx[o++] = k;
                            cnt++;
                        } else if (mark[k] == FGPT && k != i) {
                            for (int r = S->row_ptr[k]; r < S->row_ptr[k + 1]; ++r) {
                                const int h = S->col_idx[r];
                                if (mark[h] == CGPT && seen[h] != i) {
                                    seen[h] = i;
                                    if (fill) P->col_idx[o++] = h;
                                    cnt++;
                                }
                            }
                        }
                    }
                } else if (mark[i] == CGPT) {
                    cnt = 1;
                    if (fill) P->col_idx[o] = i;
                }
                if (!fill) P->row_ptr[i + 1] = cnt;
            }
        }
    }
    scratch_free(scr, T);
}

int SSS_amg_coarsen(SSS_MAT *A, SSS_IVEC *vertices, SSS_MAT *P, SSS_IMAT *S, SSS_AMG_PARS *pars)
{
    int ncoarse = 0;
    const int timing = getenv("SSS_SETUP_TIMING") != NULL;
    const double t0 = SSS_get_time();
    strong_couplings(A, S, pars);
    const double t1 = SSS_get_time();
    if (pars->cs_type == SSS_COARSE_RS) ncoarse = rs_split(A, S, vertices);
    else if (pars->cs_type != SSS_COARSE_RSP) SSS_exit_on_errcode(ERROR_AMG_COARSE_TYPE, __func__);
    if (ncoarse <= 0) return ERROR_UNKNOWN;
    const double t2 = SSS_get_time();
    if (pars->interp_type == intERP_DIR) {
        ncoarse = cleanup_ff(S, vertices, A->num_rows, ncoarse);
        const double t3 = SSS_get_time();
        direct_pattern(P, S, vertices, A->num_rows, ncoarse);
        if (timing)
            fprintf(stderr, "[setup]   coarsen: strength %.3f s, RS split %.3f s, F-F cleanup %.3f s, P pattern %.3f s\n",
                    t1 - t0, t2 - t1, t3 - t2, SSS_get_time() - t3);
    } else if (pars->interp_type == intERP_STD) {   /* no F-F cleanup before the standard pattern */
        const double t3 = SSS_get_time();
        std_pattern(P, S, vertices, A->num_rows, ncoarse);
        if (timing)
            fprintf(stderr, "[setup]   coarsen: strength %.3f s, RS split %.3f s, standard P pattern %.3f s\n", t1 - t0,
                    t2 - t1, SSS_get_time() - t3);
    } else {
        SSS_exit_on_errcode(ERROR_AMG_interp_type, __func__);
    }
    return 0;
}

/* ======================================================================================
 * Interpolation and truncation
 * ====================================================================================== */
/* Per-row form of the truncation below for large P: the same kept entries and scaled values,
 * computed row-parallel into new arrays (kept counts, prefix, fill). */
static void interp_trunc_par(SSS_MAT *P, double eps)
{
    const int n = P->num_rows;
    int *nrp = (int *)SSS_calloc((size_t)n + 1, sizeof(int));
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        const int lo = P->row_ptr[i], hi = P->row_ptr[i + 1];
        double pos_max = 0, neg_min = 0;
        int c = 0;
        for (int k = lo; k < hi; ++k) {
            double v = P->val[k];
            if (v > 0) pos_max = SSS_max(pos_max, v);
            else if (v < 0) neg_min = SSS_MIN(neg_min, v);
        }
        pos_max *= eps;
        neg_min *= eps;
        for (int k = lo; k < hi; ++k) c += (P->val[k] >= pos_max) || (P->val[k] <= neg_min);
        nrp[i + 1] = c;
    }
    for (int i = 0; i < n; ++i) nrp[i + 1] += nrp[i];
    const int kept = nrp[n];
    int *nci = (int *)SSS_calloc((size_t)(kept > 0 ? kept : 1), sizeof(int));
    double *nv = (double *)SSS_calloc((size_t)(kept > 0 ? kept : 1), sizeof(double));
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        const int lo = P->row_ptr[i], hi = P->row_ptr[i + 1];
        double pos_max = 0, neg_min = 0, pos_sum = 0, neg_sum = 0, pos_kept = 0, neg_kept = 0;
        for (int k = lo; k < hi; ++k) {
            double v = P->val[k];
            if (v > 0) { pos_sum += v; pos_max = SSS_max(pos_max, v); }
            else if (v < 0) { neg_sum += v; neg_min = SSS_MIN(neg_min, v); }
        }
        pos_max *= eps;
        neg_min *= eps;
        int o = nrp[i];
        for (int k = lo; k < hi; ++k) {
            double v = P->val[k];
            if (v >= pos_max) { nci[o++] = P->col_idx[k]; pos_kept += v; }
            else if (v <= neg_min) { nci[o++] = P->col_idx[k]; neg_kept += v; }
        }
        const double pos_fac = pos_kept > SMALLFLOAT ? pos_sum / pos_kept : 1.0;
        const double neg_fac = neg_kept < -SMALLFLOAT ? neg_sum / neg_kept : 1.0;
        o = nrp[i];
        for (int k = lo; k < hi; ++k) {
            double v = P->val[k];
            if (v >= pos_max) nv[o++] = v * pos_fac;
            else if (v <= neg_min) nv[o++] = v * neg_fac;
        }
    }
    free(P->row_ptr);
    free(P->col_idx);
    free(P->val);
    P->row_ptr = nrp;
    P->col_idx = nci;
    P->val = nv;
    P->num_nnzs = kept;
}

void SSS_amg_interp_trunc(SSS_MAT *P, SSS_AMG_PARS *pars)
{
    const double eps = pars->trunc_threshold;
    int kept = 0, wcol = 0, wval = 0;
    if (P->num_nnzs >= (1 << 20)) {
        interp_trunc_par(P, eps);
        return;
    }
    for (int i = 0; i < P->num_rows; ++i) {
        const int lo = P->row_ptr[i], hi = P->row_ptr[i + 1];
        double pos_max = 0, neg_min = 0, pos_sum = 0, neg_sum = 0, pos_kept = 0, neg_kept = 0;
        double pos_fac, neg_fac;
        P->row_ptr[i] = kept;
        for (int k = lo; k < hi; ++k) {
            double v = P->val[k];
            if (v > 0) { pos_sum += v; pos_max = SSS_max(pos_max, v); }
            else if (v < 0) { neg_sum += v; neg_min = SSS_MIN(neg_min, v); }
        }
        pos_max *= eps;
        neg_min *= eps;
        for (int k = lo; k < hi; ++k) {
            double v = P->val[k];
            if (v >= pos_max) { kept++; P->col_idx[wcol++] = P->col_idx[k]; pos_kept += v; }
            else if (v <= neg_min) { kept++; P->col_idx[wcol++] = P->col_idx[k]; neg_kept += v; }
        }
        pos_fac = pos_kept > SMALLFLOAT ? pos_sum / pos_kept : 1.0;
        neg_fac = neg_kept < -SMALLFLOAT ? neg_sum / neg_kept : 1.0;
        for (int k = lo; k < hi; ++k) {
            double v = P->val[k];
            if (v >= pos_max) P->val[wval++] = v * pos_fac;
            else if (v <= neg_min) P->val[wval++] = v * neg_fac;
        }
    }
    P->num_nnzs = P->row_ptr[P->num_rows] = kept;
    P->col_idx = (int *)SSS_realloc(P->col_idx, (size_t)kept * sizeof(int));
    P->val = (double *)SSS_realloc(P->val, (size_t)kept * sizeof(double));
}

/*
 * Setup/SSS_inter.cu:400-547.  `aii` is carried from row to row exactly as the host twin
 * does (a row without a diagonal entry reuses the previous row's value, including the
 * apN correction) — resolved up front so the weight computation can run row-parallel.
 */
void interp_DIR(SSS_MAT *A, SSS_IVEC *vertices, SSS_MAT *P, SSS_AMG_PARS *pars)
{
    const int n = A->num_rows;
    const int *mark = vertices->d;
    const int *ia = A->row_ptr, *ja = A->col_idx;
    const double *a = A->val;
    double *aii_row = (double *)sss_big_malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    int *diag_pos = (int *)sss_big_malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    int *cmap;
    double t0 = SSS_get_time(), carried = 0.0;
    int ncoarse = 0;

    /* pass 1: diagonal positions; apN corrections are needed only where the chain matters */
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        int d = ia[i + 1];
        for (int k = ia[i]; k < ia[i + 1]; ++k)
            if (ja[k] == i) { d = k; break; }
        diag_pos[i] = d;
    }
    /* pass 2: the per-row apN correction (row-parallel; stored in aii_row), then the carried aii
     * resolved in row order (a row without a diagonal entry takes the previous row's value) */
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        double apN = 0.0;
        int npos = 0, corr = 0;
        if (mark[i] == FGPT) {
            for (int k = ia[i]; k < ia[i + 1]; ++k) {
                if (k == diag_pos[i] || !(a[k] > 0)) continue;
                apN += a[k];
                for (int q = P->row_ptr[i]; q < P->row_ptr[i + 1]; ++q)
                    if (P->col_idx[q] == ja[k]) { npos++; break; }
            }
            corr = npos == 0;
        }
        aii_row[i] = apN;
        if (!corr) diag_pos[i] = -2 - diag_pos[i];   /* flag "no correction", position kept */
    }
    for (int i = 0; i < n; ++i) {
        const int corr = diag_pos[i] >= 0;
        const int d = corr ? diag_pos[i] : -2 - diag_pos[i];
        if (!corr) diag_pos[i] = d;
        double aii = d < ia[i + 1] ? a[d] : carried;
        if (corr) aii += aii_row[i];
        aii_row[i] = aii;
        carried = aii;
    }
    /* pass 3: weights, row-parallel */
#pragma omp parallel for schedule(dynamic, 4096)
    for (int i = 0; i < n; ++i) {
        const double aii = aii_row[i];
        if (mark[i] == FGPT) {
            double amN = 0.0, amP = 0.0, apN = 0.0, apP = 0.0, alpha, beta;
            int npos = 0;
            for (int k = ia[i]; k < ia[i + 1]; ++k) {
                int strong = FALSE;
                if (k == diag_pos[i]) continue;
                for (int q = P->row_ptr[i]; q < P->row_ptr[i + 1]; ++q)
                    if (P->col_idx[q] == ja[k]) { strong = TRUE; break; }
                if (a[k] > 0) {
                    apN += a[k];
                    if (strong) { apP += a[k]; npos++; }
                } else {
                    amN += a[k];
                    if (strong) amP += a[k];
                }
            }
            alpha = amN / amP;
            beta = npos > 0 ? apN / apP : 0.0;
            for (int q = P->row_ptr[i]; q < P->row_ptr[i + 1]; ++q) {
                int k = ia[i];
                while (k < ia[i + 1] && ja[k] != P->col_idx[q]) ++k;
                P->val[q] = a[k] > 0 ? -beta * a[k] / aii : -alpha * a[k] / aii;
            }
        } else if (mark[i] == CGPT) {
            P->val[P->row_ptr[i]] = 1.0;
        }
    }
    printf("-------------cpu_step1_time = %f ms -------------------\n", (SSS_get_time() - t0) * 1000.0);

    /* coarse renumbering */
    cmap = (int *)SSS_calloc((size_t)n, sizeof(int));
    for (int i = 0; i < n; ++i)
        if (mark[i] == CGPT) cmap[i] = ncoarse++;
    P->num_cols = ncoarse;
#pragma omp parallel for schedule(static)
    for (int q = 0; q < P->num_nnzs; ++q) P->col_idx[q] = cmap[P->col_idx[q]];
    free(cmap);
    free(aii_row);
    free(diag_pos);
    SSS_amg_interp_trunc(P, pars);
}

/*
 * Setup/SSS_inter.cu:550-715 (interp_STD), on the pattern std_pattern built.  Per F row i, with
 * hat a the row's entries eliminated through its strong F neighbours k:
 *   hat a_ii = a_ii - sum_k (a_ik / a_kk) a_ki,   hat a_il = a_il [l in C_i^s] - sum_k (a_ik / a_kk) a_kl [l in C_k^s]
 *   alpha = (psum_i - sum_k f_k (nsum_k - a_ki + a_kk)) / (csum_i - sum_k f_k csum_k),
 *   p_il = -alpha hat a_il / hat a_ii
 * (psum: off-diagonal entries whose column is not isolated; nsum: all off-diagonal entries; csum:
 * the entries of strong C neighbours; every sum in stored order).  The reference's per-row scratch
 * (reverse indices of rows i and k, hat a) is reset or fully rewritten for each row before it is
 * read, so the rows are computed in parallel with per-thread scratch; each row's arithmetic is the
 * reference's, in its order.  (The reference also sets the process's OpenMP thread count to 8 here,
 * a speed-only side effect not reproduced.)  Then the coarse renumbering and the truncation.
 */
static void interp_STD(SSS_MAT *A, SSS_IVEC *vertices, SSS_MAT *P, SSS_IMAT *S, SSS_AMG_PARS *pars)
{
    const int n = A->num_rows, nc = A->num_cols > n ? A->num_cols : n;
    const int *mark = vertices->d;
    const int *ia = A->row_ptr, *ja = A->col_idx;
    const double *a = A->val;
    double *csum = (double *)SSS_calloc((size_t)(n > 0 ? n : 1), sizeof(double));
    double *psum = (double *)SSS_calloc((size_t)(n > 0 ? n : 1), sizeof(double));
    double *nsum = (double *)SSS_calloc((size_t)(n > 0 ? n : 1), sizeof(double));
    double *diag = (double *)SSS_calloc((size_t)(n > 0 ? n : 1), sizeof(double));

    /* step 0: diagonal (the row's last diagonal entry), strong-C, off-diagonal and non-isolated sums */
#pragma omp parallel for schedule(dynamic, 4096) if (n > 65536)
    for (int i = 0; i < n; ++i) {
        double cs = 0.0, ns = 0.0, ps = 0.0, d = 0.0;
        for (int j = ia[i]; j < ia[i + 1]; ++j) {
            const int k = ja[j];
            int strong_c = 0;
            if (mark[k] == CGPT)
                for (int q = S->row_ptr[i]; q < S->row_ptr[i + 1] && !strong_c; ++q) strong_c = S->col_idx[q] == k;
            if (strong_c) cs += a[j];
            if (k == i) {
                d = a[j];
            } else {
                ns += a[j];
                if (mark[k] != ISPT) ps += a[j];
            }
        }
        csum[i] = cs, nsum[i] = ns, psum[i] = ps, diag[i] = d;
    }

    /* step 1: the weights */
    /* per thread: rindi and rindk (ints) and ahat (doubles), nc each, in one buffer */
    void *scr[kScratchMax];
    const size_t ncs = (size_t)(nc > 0 ? nc : 1);
    const int T = scratch_alloc(ncs * (2 * sizeof(int) + sizeof(double)), scr);
#pragma omp parallel num_threads(T) if (n > 4096)
    {
        double *ahat = (double *)scr[omp_get_thread_num()];
        int *rindi = (int *)(ahat + ncs), *rindk = rindi + ncs;
#pragma omp for schedule(dynamic, 1024)
        for (int i = 0; i < n; ++i) {
            if (mark[i] == CGPT) {
                P->val[P->row_ptr[i]] = 1.0;
                continue;
            }
            if (mark[i] != FGPT) continue;
            double alN = psum[i], alP = csum[i], alpha = 0.0;
            for (int j = ia[i]; j < ia[i + 1]; ++j) rindi[ja[j]] = j;
            for (int j = P->row_ptr[i]; j < P->row_ptr[i + 1]; ++j) ahat[P->col_idx[j]] = 0.0;
            ahat[i] = diag[i];
            for (int j = S->row_ptr[i]; j < S->row_ptr[i + 1]; ++j) {
                const int k = S->col_idx[j];
                const double aik = a[rindi[k]];
                if (mark[k] == CGPT) {
                    ahat[k] += aik;
                } else if (mark[k] == FGPT) {
                    const double akk = diag[k];
                    for (int m = ia[k]; m < ia[k + 1]; ++m) rindk[ja[m]] = m;
                    const double factor = aik / akk;
                    double aki = 0.0;
                    for (int m = ia[k]; m < ia[k + 1]; ++m)
                        if (ja[m] == i) {
                            aki = a[m];
                            ahat[i] -= factor * aki;
                        }
                    for (int m = S->row_ptr[k]; m < S->row_ptr[k + 1]; ++m) {
                        const int l = S->col_idx[m];
                        const double akl = a[rindk[l]];
                        if (mark[l] == CGPT) ahat[l] -= factor * akl;
                    }
                    alN -= factor * (nsum[k] - aki + akk);
                    alP -= factor * csum[k];
                }
            }
            if (P->row_ptr[i + 1] > P->row_ptr[i]) alpha = alN / alP;
            for (int j = P->row_ptr[i]; j < P->row_ptr[i + 1]; ++j) P->val[j] = -alpha * ahat[P->col_idx[j]] / ahat[i];
        }
    }
    scratch_free(scr, T);

    /* step 2: coarse renumbering of the columns */
    int *cmap = (int *)SSS_calloc((size_t)(n > 0 ? n : 1), sizeof(int));
    int ncoarse = 0;
    for (int i = 0; i < n; ++i)
        if (mark[i] == CGPT) cmap[i] = ncoarse++;
    P->num_cols = ncoarse;
#pragma omp parallel for schedule(static) if (P->num_nnzs > 65536)
    for (int q = 0; q < P->row_ptr[P->num_rows]; ++q) P->col_idx[q] = cmap[P->col_idx[q]];
    free(cmap);
    free(csum);
    free(psum);
    free(nsum);
    free(diag);
    /* step 3 */
    SSS_amg_interp_trunc(P, pars);
}

void SSS_amg_interp(SSS_MAT *A, SSS_IVEC *vertices, SSS_MAT *P, SSS_IMAT *S, SSS_AMG_PARS *pars)
{
    if (pars->interp_type == intERP_DIR) interp_DIR(A, vertices, P, pars);
    else if (pars->interp_type == intERP_STD) interp_STD(A, vertices, P, S, pars);
    else SSS_exit_on_errcode(ERROR_AMG_interp_type, __func__);
}

/* ======================================================================================
 * Galerkin product A_c = R A P (SSS_matvec.c:398-534), row-parallel.
 * ====================================================================================== */
SSS_MAT SSS_blas_mat_rap(const SSS_MAT *R, const SSS_MAT *A, const SSS_MAT *P)
{
    const int nc = R->num_rows, nf = A->num_rows;
    const int *ri = R->row_ptr, *rj = R->col_idx, *ai = A->row_ptr, *aj = A->col_idx;
    const int *pi = P->row_ptr, *pj = P->col_idx;
    const double *rv = R->val, *av = A->val, *pv = P->val;
    int64_t *start = (int64_t *)sss_big_calloc((size_t)nc + 1, sizeof(int64_t));
    SSS_MAT C;
    int too_big = 0;

    C.num_rows = nc;
    C.num_cols = nc;
    C.row_ptr = (int *)SSS_calloc((size_t)nc + 1, sizeof(int));
    C.col_idx = NULL;
    C.val = NULL;
    C.num_nnzs = 0;

    /* One parallel region for both passes: each thread's marker arrays are initialised once.
     * Markers hold the coarse row being built: ic in the counting pass, nc + ic in the filling
     * pass, so the second pass needs no reset. */
#pragma omp parallel
    {
        int *seen_f = (int *)sss_big_malloc(sizeof(int) * (size_t)(nf > 0 ? nf : 1));
        int *seen_c = (int *)sss_big_malloc(sizeof(int) * (size_t)(nc > 0 ? nc : 1));
        int *slot = (int *)sss_big_malloc(sizeof(int) * (size_t)(nc > 0 ? nc : 1));
        for (int i = 0; i < nf; ++i) seen_f[i] = -1;
        for (int i = 0; i < nc; ++i) seen_c[i] = -1;
#pragma omp for schedule(dynamic, 256)
        for (int ic = 0; ic < nc; ++ic) {
            int64_t cnt = 1;
            seen_c[ic] = ic;
            for (int q1 = ri[ic]; q1 < ri[ic + 1]; ++q1) {
                int i1 = rj[q1];
                for (int q2 = ai[i1]; q2 < ai[i1 + 1]; ++q2) {
                    int i2 = aj[q2];
                    if (seen_f[i2] == ic) continue;
                    seen_f[i2] = ic;
                    for (int q3 = pi[i2]; q3 < pi[i2 + 1]; ++q3)
                        if (seen_c[pj[q3]] != ic) { seen_c[pj[q3]] = ic; cnt++; }
                }
            }
            start[ic + 1] = cnt;
        }
#pragma omp single
        {
            for (int ic = 0; ic < nc; ++ic) start[ic + 1] += start[ic];
            if (start[nc] > INT32_MAX) {
                too_big = 1;
            } else {
                C.num_nnzs = (int)start[nc];
                for (int ic = 0; ic <= nc; ++ic) C.row_ptr[ic] = (int)start[ic];
                C.col_idx = (int *)SSS_calloc((size_t)C.num_nnzs, sizeof(int));
                C.val = (double *)SSS_calloc((size_t)C.num_nnzs, sizeof(double));
            }
        }   /* implicit barrier */
        if (!too_big) {
#pragma omp for schedule(dynamic, 256)
            for (int ic = 0; ic < nc; ++ic) {
                const int mk = nc + ic;
                int pos = C.row_ptr[ic];
                seen_c[ic] = mk;
                slot[ic] = pos;
                C.col_idx[pos] = ic;
                C.val[pos] = 0.0;
                pos++;
                for (int q1 = ri[ic]; q1 < ri[ic + 1]; ++q1) {
                    const double r = rv[q1];
                    const int i1 = rj[q1];
                    for (int q2 = ai[i1]; q2 < ai[i1 + 1]; ++q2) {
                        const double ra = r * av[q2];
                        const int i2 = aj[q2];
                        if (seen_f[i2] != mk) {
                            seen_f[i2] = mk;
                            for (int q3 = pi[i2]; q3 < pi[i2 + 1]; ++q3) {
                                const double rap = ra * pv[q3];
                                const int i3 = pj[q3];
                                if (seen_c[i3] != mk) {
                                    seen_c[i3] = mk;
                                    slot[i3] = pos;
                                    C.val[pos] = rap;
                                    C.col_idx[pos] = i3;
                                    pos++;
                                } else {
                                    C.val[slot[i3]] += rap;
                                }
                            }
                        } else {
                            for (int q3 = pi[i2]; q3 < pi[i2 + 1]; ++q3) C.val[slot[pj[q3]]] += ra * pv[q3];
                        }
                    }
                }
            }
        }
        free(seen_f);
        free(seen_c);
        free(slot);
    }
    if (too_big) {
        printf("### ERROR: RAP product has %lld nonzeros (int32 index limit)\n", (long long)start[nc]);
        SSS_exit_on_errcode(ERROR_MAT_SIZE, __func__);
    }
    free(start);
    return C;
}

/* ======================================================================================
 * Level loop (Setup/SSS_SETUP.cu:5-178)
 * ====================================================================================== */
void SSS_amg_complexity_print(SSS_AMG *mg)
{
    static const char *rule = "-----------------------------------------------------------\n";
    double grid = 0.0, op = 0.0;
    fputs(rule, stdout);
    printf("  Level   Num of rows   Num of nonzeros   Avg. NNZ / row   \n");
    fputs(rule, stdout);
    for (int l = 0; l < mg->num_levels; ++l) {
        const SSS_MAT *A = &mg->cg[l].A;
        printf("%5d %13d %17d %14.2lf\n", l, A->num_rows, A->num_nnzs, (double)A->num_nnzs / A->num_rows);
        grid += A->num_rows;
        op += A->num_nnzs;
    }
    fputs(rule, stdout);
    grid /= mg->cg[0].A.num_rows;
    op /= mg->cg[0].A.num_nnzs;
    printf("  Grid complexity = %.3lf  |", grid);
    printf("  Operator complexity = %.3lf\n", op);
    fputs(rule, stdout);
}

void SSS_amg_setup(SSS_AMG *mg, SSS_MAT *A, SSS_AMG_PARS *pars) { sss_amg_setup_hooked(mg, A, pars, NULL, NULL); }

/* SSS_amg_setup with a progress hook: hook(ctx, mg, done, 0) each time level done - 1 has been
 * completed (its P, R, C/F marks and the next operator are final and it is not the coarsest
 * level), hook(ctx, mg, num_levels - 1, 1) at the end.  sss_hip_setup_create uploads the
 * completed levels to the GPU while the later ones are still being coarsened. */
void sss_amg_setup_hooked(SSS_AMG *mg, SSS_MAT *A, SSS_AMG_PARS *pars, sss_setup_hook hook, void *ctx)
{
    const int min_cdof = SSS_max(pars->coarse_dof, MIN_CDOF);
    const int max_lvls = pars->max_levels;
    const int n0 = A->num_rows;
    const double t0 = SSS_get_time();
    SSS_IVEC vertices;
    int lvl = 0;
    /* the Galerkin products of the large levels on the GPU when one is present (same result) */
    const char *gr = getenv("SSS_SETUP_GPU_RAP"), *grm = getenv("SSS_SETUP_GPU_RAP_MIN");
    const int use_gpu_rap = !(gr && gr[0] == '0') && sss_hip_device_count() > 0;
    const int gpu_rap_min = (grm && *grm) ? atoi(grm) : 1000000;
    const char *grx = getenv("SSS_SETUP_GPU_RAP_MAXROW");   /* average A row length up to which */
    const int gpu_rap_maxrow = (grx && *grx) ? atoi(grx) : 48;

    *mg = SSS_amg_data_create(pars);
    vertices = SSS_ivec_create(n0);
    mg->cg[0].A = SSS_mat_struct_create(n0, n0, A->num_nnzs);
    SSS_mat_cp(A, &mg->cg[0].A);

    while (mg->cg[lvl].A.num_rows > min_cdof && lvl < max_lvls - 1) {
        SSS_AMG_COMP *L = &mg->cg[lvl];
        SSS_IMAT S;
        int status;
        memset(&S, 0, sizeof(S));

        const double tc0 = SSS_get_time();
        sss_trace_push("SSS_amg_setup level %d", lvl);
        sss_trace_push("coarsen");
        status = SSS_amg_coarsen(&L->A, &vertices, &L->P, &S, pars);
        sss_trace_pop();
        const double tc1 = SSS_get_time();
        if (status < 0) {
            free(S.row_ptr);
            free(S.col_idx);
            printf("### WARNING: Could not find any C-variables!\n");
            printf("### WARNING: RS coarsening on level-%d failed!\n", lvl);
            sss_trace_pop();
            break;
        }
        if (L->P.num_cols < min_cdof) {
            free(S.row_ptr);
            free(S.col_idx);
            sss_trace_pop();
            break;
        }
        if (L->P.num_rows > L->P.num_cols * 10) {
            printf("### WARNING: Coarsening might be too aggressive!\n");
            printf("### WARNING: Lvl = %d ,Fine level = %d, coarse level = %d. Discard!\n", lvl,
                   L->P.num_rows, L->P.num_cols);
        }
        if (L->P.num_cols * 1.5 > L->A.num_rows) pars->cs_type = SSS_COARSE_RS;

        L->cfmark = SSS_ivec_create(L->A.num_rows);
        memcpy(L->cfmark.d, vertices.d, (size_t)L->A.num_rows * sizeof(int));

        sss_trace_push("interpolation");
        SSS_amg_interp(&L->A, &vertices, &L->P, &S, pars);
        sss_trace_pop();
        const double tc2 = SSS_get_time();
        sss_trace_push("R = P^T");
        L->R = SSS_mat_trans(&L->P);
        sss_trace_pop();
        const double tc3 = SSS_get_time();
        sss_trace_push("RAP");
        /* the device walks each coarse row's (R entry, A entry) steps in order, so it wins on the
         * wide levels of short rows (7-pt 400^3 levels 0-2: 3.1 -> 1.1, 2.0 -> 0.75, 0.59 -> 0.37 s)
         * and loses on the narrow levels of long rows (level 3 and below: 0.75 -> 1.2 s) */
        const int gpu_here = use_gpu_rap && L->A.num_nnzs >= gpu_rap_min &&
                             (double)L->A.num_nnzs <= (double)gpu_rap_maxrow * L->A.num_rows;
        if (!(gpu_here && sss_hip_rap(&L->R, &L->A, &L->P, &mg->cg[lvl + 1].A) == 0))
            mg->cg[lvl + 1].A = SSS_blas_mat_rap(&L->R, &L->A, &L->P);
        sss_trace_pop();
        sss_trace_pop();   /* the level */
        if (getenv("SSS_SETUP_TIMING"))   /* phase times on stderr (stdout stays the reference's) */
            fprintf(stderr, "[setup] level %d: coarsen %.3f s, interp %.3f s, transpose %.3f s, RAP %.3f s\n", lvl,
                    tc1 - tc0, tc2 - tc1, tc3 - tc2, SSS_get_time() - tc3);
        free(S.row_ptr);
        free(S.col_idx);

        /* "too dense" test on the finer level (integer nnz/rows, SSS_SETUP.cu:142) */
        if (L->A.num_nnzs / L->A.num_rows > L->A.num_cols * 0.2) {
            printf("### WARNING: Coarse matrix is too dense!\n");
            printf("### WARNING: m = n = %d, nnz = %d!\n", L->A.num_cols, L->A.num_nnzs);
            SSS_mat_destroy(&mg->cg[lvl + 1].A);
            break;
        }
        lvl++;
        if (hook) hook(ctx, mg, lvl, 0);
    }

    mg->num_levels = lvl + 1;
    mg->cg[0].wp = SSS_vec_create(n0);
    for (int l = 1; l < mg->num_levels; ++l) {
        int m = mg->cg[l].A.num_rows;
        mg->cg[l].b = SSS_vec_create(m);
        mg->cg[l].x = SSS_vec_create(m);
        mg->cg[l].wp = SSS_vec_create(2 * m);
    }
    SSS_ivec_destroy(&vertices);
    SSS_amg_complexity_print(mg);
    printf("AMG setup time: %g s\n", SSS_get_time() - t0);
    if (hook) hook(ctx, mg, mg->num_levels - 1, 1);
}
