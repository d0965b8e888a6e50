/*
 * ref_cycle_glue.c — TEST INFRASTRUCTURE ONLY (linked into oracle/_ref/libsss_ref.so, never into
 * the product).
 *
 * The reference's outer loop SSS_amg_solve (Solve/SSS_SOLVE.c:4-87) is pure C and builds here, but
 * the SSS_amg_cycle it calls (Solve/SSS_SOLVE.c:56) lives in Solve/SSS_cycle.cu, which includes
 * <cuda.h> and is unbuildable in this image.  This resolves that one call to the oracle's restated
 * cycle (oracle/sss_oracle.c ora_cycle, reference semantics: GS-CF, CG(beta==1)+GMRES coarse
 * solve), so the reference's own loop, stop test, rtn bookkeeping and iteration print can be run
 * and compared with the product's SSS_amg_solve (tests/test_ref_units.py).
 */
#include "sss_oracle.h"

void SSS_amg_cycle(SSS_AMG *mg)
{
    ora_opts o;
    ora_opts_default(&o);
    ora_cycle(mg, &o);
}
