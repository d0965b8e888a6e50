/*
 * sss_hierio.c — binary file format for a set-up AMG hierarchy ("hierarchy
 * file format ... 512^3 cannot be a text file").  Engine extension; host C.
 *
 * The host setup (Setup/SSS_SETUP.cu:36 semantics, amg_amd/host/sss_setup.c) takes ~46 s at 400^3,
 * 3 orders of magnitude above a V-cycle.  SSS_amg_save writes everything the solve phase reads --
 * parameters, and per level A, P, R (CSR) and the C/F marker -- and SSS_amg_load rebuilds an
 * SSS_AMG that is field-for-field the one SSS_amg_setup produced (the solve phase's vectors b, x,
 * wp are allocated as the setup allocates them), so every later result is bitwise the same.
 *
 * Layout (little-endian, native LP64 types):
 *   "SSSAMG01"  int32 version=1  int32 num_levels  int32 sizeof(SSS_AMG_PARS)  SSS_AMG_PARS
 *   per level l:  matrix A_l;  l < num_levels-1: matrix P_l, matrix R_l, int32 n + n int32 cfmark
 *   matrix := int32 rows, cols, nnz; (rows+1) int32 row_ptr; nnz int32 col_idx; nnz float64 val
 * Errors return ERROR_OPEN_FILE / ERROR_WRONG_FILE (SSS_main.h codes); nothing is printed.
 */
#include "../../include/sss_amg.h"
#include "../../include/sss_hip.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const char kMagic[8] = {'S', 'S', 'S', 'A', 'M', 'G', '0', '1'};

static int put(FILE *f, const void *p, size_t bytes) { return bytes == 0 || fwrite(p, 1, bytes, f) == bytes ? 0 : -1; }
static int get(FILE *f, void *p, size_t bytes) { return bytes == 0 || fread(p, 1, bytes, f) == bytes ? 0 : -1; }

static int put_mat(FILE *f, const SSS_MAT *A)
{
    const int32_t h[3] = {A->num_rows, A->num_cols, A->num_nnzs};
    if (put(f, h, sizeof(h))) return -1;
    if (put(f, A->row_ptr, sizeof(int) * ((size_t)A->num_rows + 1))) return -1;
    if (put(f, A->col_idx, sizeof(int) * (size_t)A->num_nnzs)) return -1;
    return put(f, A->val, sizeof(double) * (size_t)A->num_nnzs);
}

static int get_mat(FILE *f, SSS_MAT *A)
{
    int32_t h[3];
    if (get(f, h, sizeof(h)) || h[0] < 0 || h[1] < 0 || h[2] < 0) return -1;
    *A = SSS_mat_struct_create(h[0], h[1], h[2]);
    if (get(f, A->row_ptr, sizeof(int) * ((size_t)h[0] + 1))) return -1;
    if (get(f, A->col_idx, sizeof(int) * (size_t)h[2])) return -1;
    if (get(f, A->val, sizeof(double) * (size_t)h[2])) return -1;
    return A->row_ptr[h[0]] == h[2] ? 0 : -1;
}

int SSS_amg_save(const SSS_AMG *mg, const char *path)
{
    FILE *f = fopen(path, "wb");
    if (!f) return ERROR_OPEN_FILE;
    const int32_t head[3] = {1, mg->num_levels, (int32_t)sizeof(SSS_AMG_PARS)};
    int bad = put(f, kMagic, sizeof(kMagic)) || put(f, head, sizeof(head)) || put(f, &mg->pars, sizeof(mg->pars));
    for (int l = 0; l < mg->num_levels && !bad; ++l) {
        const SSS_AMG_COMP *L = &mg->cg[l];
        bad = put_mat(f, &L->A);
        if (!bad && l + 1 < mg->num_levels) {
            const int32_t n = L->cfmark.n;
            bad = put_mat(f, &L->P) || put_mat(f, &L->R) || put(f, &n, sizeof(n)) ||
                  put(f, L->cfmark.d, sizeof(int) * (size_t)n);
        }
    }
    if (fclose(f) != 0) bad = 1;
    return bad ? ERROR_OPEN_FILE : 0;
}

int SSS_amg_load(SSS_AMG *mg, const char *path)
{
    FILE *f = fopen(path, "rb");
    char magic[8];
    int32_t head[3];
    SSS_AMG_PARS pars;
    if (!f) return ERROR_OPEN_FILE;
    memset(mg, 0, sizeof(*mg));
    if (get(f, magic, sizeof(magic)) || memcmp(magic, kMagic, sizeof(magic)) || get(f, head, sizeof(head)) ||
        head[0] != 1 || head[2] != (int32_t)sizeof(SSS_AMG_PARS) || get(f, &pars, sizeof(pars)) || head[1] < 1 ||
        head[1] > pars.max_levels) {
        fclose(f);
        return ERROR_WRONG_FILE;
    }
    *mg = SSS_amg_data_create(&pars);
    mg->num_levels = head[1];
    int bad = 0;
    for (int l = 0; l < mg->num_levels && !bad; ++l) {
        SSS_AMG_COMP *L = &mg->cg[l];
        bad = get_mat(f, &L->A);
        if (!bad && l + 1 < mg->num_levels) {
            int32_t n;
            bad = get_mat(f, &L->P) || get_mat(f, &L->R) || get(f, &n, sizeof(n)) || n != L->A.num_rows;
            if (!bad) {
                L->cfmark = SSS_ivec_create(n);
                bad = get(f, L->cfmark.d, sizeof(int) * (size_t)n);
            }
        }
    }
    fclose(f);
    if (bad) {
        SSS_amg_data_destroy(mg);
        return ERROR_WRONG_FILE;
    }
    /* the solve phase's work vectors, exactly as SSS_amg_setup allocates them */
    mg->cg[0].wp = SSS_vec_create(mg->cg[0].A.num_rows);
    for (int l = 1; l < mg->num_levels; ++l) {
        const int m = mg->cg[l].A.num_rows;
        mg->cg[l].b = SSS_vec_create(m);
        mg->cg[l].x = SSS_vec_create(m);
        mg->cg[l].wp = SSS_vec_create(2 * m);
    }
    return 0;
}
