/* dag_depths.c -- lab tool: per level of a 7-/27-pt hierarchy, the exact GS-CF pass structure
 * (rows, same-class couplings, level-schedule depth of the F and C passes, widest depth) and the
 * greedy distance-1 colour count of each class's coupling graph.  Host only.
 *
 *   gcc -O2 -fopenmp -Iinclude tools/dag_depths.c -Lamg_amd/lib -lsss_amg -Wl,-rpath,$PWD/amg_amd/lib -o /tmp/dag_depths
 *   /tmp/dag_depths 7 128
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sss_amg.h"
#include "sss_hip.h"

static int imax(int a, int b) { return a > b ? a : b; }

int main(int argc, char **argv)
{
    int kind = argc > 1 ? atoi(argv[1]) : 7, n = argc > 2 ? atoi(argv[2]) : 64;
    SSS_MAT A;
    if (sss_gen_stencil(kind, n, n, n, 0, n, &A)) return 1;
    SSS_AMG_PARS pars;
    SSS_amg_pars_init(&pars);
    SSS_AMG mg;
    memset(&mg, 0, sizeof mg);
    SSS_amg_setup(&mg, &A, &pars);
    long long tot_depth = 0;
    printf("level rows nnz | F: rows depth maxw same-class-nnz colours | C: rows depth maxw same-class-nnz colours\n");
    for (int l = 0; l + 1 < mg.num_levels; ++l) {
        SSS_MAT *M = &mg.cg[l].A;
        const int m = M->num_rows, *rp = M->row_ptr, *ci = M->col_idx;
        const int *mark = mg.cg[l].cfmark.d;
        int *cls = malloc(sizeof(int) * m), *dep = calloc(m, sizeof(int)), *push = calloc(m, sizeof(int));
        int *col = malloc(sizeof(int) * m);
        for (int i = 0; i < m; ++i) cls[i] = mark[i] == 1;
        for (int i = 0; i < m; ++i) {
            int d = push[i];
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                int j = ci[k];
                if (j < i && cls[j] == cls[i]) d = imax(d, dep[j] + 1);
            }
            dep[i] = d;
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                int j = ci[k];
                if (j > i && cls[j] == cls[i] && push[j] < d + 1) push[j] = d + 1;
            }
        }
        /* greedy colouring of each class's coupling graph in row order */
        int maxc = 4096;
        char *used = calloc(maxc, 1);
        for (int i = 0; i < m; ++i) {
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                int j = ci[k];
                if (j < i && cls[j] == cls[i]) used[col[j]] = 1;
            }
            /* symmetric patterns: neighbours j > i are coloured later and avoid i */
            int c = 0;
            while (used[c]) ++c;
            col[i] = c;
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                int j = ci[k];
                if (j < i && cls[j] == cls[i]) used[col[j]] = 0;
            }
        }
        printf("%2d %9d %10d |", l, m, rp[m]);
        for (int c = 0; c < 2; ++c) {
            int rows = 0, depth = 0, colours = 0;
            long long same = 0;
            int *w = calloc(m + 1, sizeof(int));
            for (int i = 0; i < m; ++i) {
                if (cls[i] != c) continue;
                ++rows;
                depth = imax(depth, dep[i] + 1);
                colours = imax(colours, col[i] + 1);
                w[dep[i]]++;
                for (int k = rp[i]; k < rp[i + 1]; ++k)
                    if (ci[k] != i && cls[ci[k]] == c) ++same;
            }
            int maxw = 0;
            for (int d = 0; d < depth; ++d) maxw = imax(maxw, w[d]);
            printf(" %8d %6d %7d %10lld %4d |", rows, depth, maxw, same, colours);
            tot_depth += depth;
            free(w);
        }
        printf("\n");
        free(cls), free(dep), free(push), free(col), free(used);
    }
    printf("sum of pass depths over levels (one sweep): %lld\n", tot_depth);
    return 0;
}
