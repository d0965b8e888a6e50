/*
 * sss_poisson.c — in-memory generators for the BASELINE problems.
 *
 * A 400^3 or 512^3 operator cannot go through a text .mtx file (~120 GB), so the bench and
 * the tests build the CSR directly.  The result is exactly the CSR mmio_data
 * (mmio_highlevel.h:144-305) produces from a row-ordered "general" .mtx of the same operator:
 * unknown (i,j,k) -> row i + nx*(j + ny*k), columns ascending inside each row.
 *
 *   7-pt  : diagonal 6, -1 to each in-grid face neighbour (Dirichlet: off-grid dropped).
 *   27-pt : diagonal 9.8 (= 8 + 18*0.1, constant), -1 to the 8 in-plane neighbours,
 *           -0.1 to the 18 neighbours with dz = +-1 (anisotropic).
 *
 * Rows [z0*nx*ny, z1*nx*ny) of the global grid are generated (a z-slab, as one rank of the
 * row partition owns); column indices stay global.
 */
#include "sss_internal.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int stencil_row(int kind, int nx, int ny, int nz, int64_t row, int *cols, double *vals)
{
    const int i = (int)(row % nx), j = (int)((row / nx) % ny), k = (int)(row / ((int64_t)nx * ny));
    int cnt = 0;
    if (kind == 7) {
        static const int off[7][3] = {{0, 0, -1}, {0, -1, 0}, {-1, 0, 0}, {0, 0, 0},
                                      {1, 0, 0},  {0, 1, 0},  {0, 0, 1}};
        for (int s = 0; s < 7; ++s) {
            int ii = i + off[s][0], jj = j + off[s][1], kk = k + off[s][2];
            if (ii < 0 || ii >= nx || jj < 0 || jj >= ny || kk < 0 || kk >= nz) continue;
            cols[cnt] = ii + nx * (jj + ny * kk);
            vals[cnt] = (s == 3) ? 6.0 : -1.0;
            cnt++;
        }
        return cnt;
    }
    for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                int ii = i + dx, jj = j + dy, kk = k + dz;
                if (ii < 0 || ii >= nx || jj < 0 || jj >= ny || kk < 0 || kk >= nz) continue;
                cols[cnt] = ii + nx * (jj + ny * kk);
                if (dx == 0 && dy == 0 && dz == 0) vals[cnt] = 9.8;
                else vals[cnt] = (dz == 0) ? -1.0 : -0.1;
                cnt++;
            }
    return cnt;
}

/* Returns 0 on success, ERROR_MAT_SIZE if the slab would overflow int32 indices. */
int sss_gen_stencil(int kind, int nx, int ny, int nz, int z0, int z1, SSS_MAT *A)
{
    const int64_t plane = (int64_t)nx * ny;
    const int64_t r0 = (int64_t)z0 * plane, r1 = (int64_t)z1 * plane;
    const int64_t nrows = r1 - r0;
    const int64_t ncols = plane * nz;
    int64_t nnz = 0;
    int *rp;

    if ((kind != 7 && kind != 27) || nrows <= 0 || ncols > INT32_MAX) return ERROR_MAT_SIZE;
    rp = (int *)sss_big_malloc(sizeof(int) * (size_t)(nrows + 1));
    rp[0] = 0;
    /* row lengths depend only on the boundary position: count in parallel, scan serially */
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < nrows; ++r) {
        int cols[27];
        double vals[27];
        rp[r + 1] = stencil_row(kind, nx, ny, nz, r0 + r, cols, vals);
    }
    for (int64_t r = 0; r < nrows; ++r) {
        nnz += rp[r + 1];
        if (nnz > INT32_MAX) { free(rp); return ERROR_MAT_SIZE; }
        rp[r + 1] = (int)nnz;
    }
    A->num_rows = (int)nrows;
    A->num_cols = (int)ncols;
    A->num_nnzs = (int)nnz;
    A->row_ptr = rp;
    A->col_idx = (int *)sss_big_malloc(sizeof(int) * (size_t)(nnz > 0 ? nnz : 1));
    A->val = (double *)sss_big_malloc(sizeof(double) * (size_t)(nnz > 0 ? nnz : 1));
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < nrows; ++r)
        stencil_row(kind, nx, ny, nz, r0 + r, A->col_idx + rp[r], A->val + rp[r]);
    return 0;
}
