/*
 * sss_main.c — the `amg` command line driver (SSS_main.c:121-160, same behaviour and stdout).
 *
 *   ./amg file.mtx          reads the .mtx, default parameters, b = x = 1, SSS_solver_amg
 *
 * Engine knobs are environment variables (the CLI itself stays identical to the reference's):
 * SSS_HIP_SMOOTHER, SSS_HIP_COARSE, SSS_HIP_ROWCAP, SSS_HIP_DEVICE (see include/sss_hip.h).
 * Extension for inputs too large for a text file: SSS_GEN=poisson7:N or aniso27:N builds the
 * operator in memory instead of reading argv[1].
 */
#include "sss_internal.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int generate(const char *spec, SSS_MAT *A)
{
    int n = 0, kind = 0;
    if (sscanf(spec, "poisson7:%d", &n) == 1) kind = 7;
    else if (sscanf(spec, "aniso27:%d", &n) == 1) kind = 27;
    if (!kind || n <= 0) return -1;
    printf("generated: %s\n", spec);
    if (sss_gen_stencil(kind, n, n, n, 0, n, A) != 0) return -1;
    printf("A: m = %d, n = %d, nnz = %d\n", A->num_rows, A->num_cols, A->num_nnzs);
    return 0;
}

int main(int argc, char *argv[])
{
    SSS_AMG_PARS pars;
    SSS_MAT A;
    SSS_VEC b, x;
    SSS_RTN rtn;
    const char *gen = getenv("SSS_GEN");

    if (gen && *gen) {
        if (generate(gen, &A) != 0) SSS_exit_on_errcode(ERROR_INPUT_PAR, "main");
    } else {
        if (argc < 2) {
            fprintf(stderr, "usage: %s matrix.mtx\n", argv[0]);
            return ERROR_INPUT_PAR;
        }
        SSS_mat_read(argv[1], &A);
    }
    SSS_amg_pars_init(&pars);
    SSS_amg_pars_print(&pars);

    b = SSS_vec_create(A.num_rows);
    SSS_vec_set_value(&b, 1.0);
    x = SSS_vec_create(A.num_rows);
    SSS_vec_set_value(&x, 1.0);

    rtn = SSS_solver_amg(&A, &x, &b, &pars);

    printf("AMG residual: %g\n", rtn.ares);
    printf("AMG relative residual: %g\n", rtn.rres);
    printf("AMG iterations: %d\n", rtn.nits);

    SSS_mat_destroy(&A);
    SSS_vec_destroy(&x);
    SSS_vec_destroy(&b);
    return 0;
}
