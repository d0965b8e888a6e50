"""TEST INFRASTRUCTURE ONLY — ctypes loaders for the parity checkers.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package;
the product (amg_amd/, libsss_amg.so) never does.

  load()      -> oracle/liboracle.so: CPU restatement of the reference solve phase
  load_ref()  -> oracle/_ref/libsss_ref.so: the reference's own pure-C units (only where the
                 reference tree was present at build time; None otherwise)
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

from amg_amd._native import SSS_AMG, SSS_IMAT, SSS_IVEC, SSS_KRYLOV, SSS_MAT, SSS_RTN, SSS_SMTR, SSS_VEC

HERE = Path(__file__).resolve().parent
ORACLE_PATH = HERE / "liboracle.so"
REF_PATH = HERE / "_ref" / "libsss_ref.so"


class ORA_OPTS(C.Structure):
    _fields_ = [("row_cap", C.c_int), ("coarse_mode", C.c_int), ("smoother", C.c_int), ("jacobi_from", C.c_int),
                ("verbose", C.c_int),
                ("jacobi_l1", C.c_int), ("omega", C.c_double), ("inner", C.c_int),
                ("inner_mask", C.c_int), ("inner_long", C.c_int), ("long_mask", C.c_int)]


_ora = None
_ref = None


def load():
    global _ora
    if _ora is None:
        if not ORACLE_PATH.exists():
            raise RuntimeError(f"{ORACLE_PATH} missing: run `make oracle`")
        lib = C.CDLL(str(ORACLE_PATH))
        P = C.POINTER
        dp, ip = P(C.c_double), P(C.c_int)
        sigs = {
            "ora_opts_default": (None, [P(ORA_OPTS)]),
            "ora_set_threads": (None, [C.c_int]),
            "ora_get_threads": (C.c_int, []),
            "ora_mv_amxpy": (None, [C.c_double, P(SSS_MAT), dp, dp, C.c_int]),
            "ora_mv_mxy": (None, [P(SSS_MAT), dp, dp]),
            "ora_mv_acc": (None, [P(SSS_MAT), dp, dp, C.c_int]),
            "ora_gs_cf": (None, [dp, P(SSS_MAT), dp, C.c_int, ip, C.c_int]),
            "ora_gs": (None, [dp, C.c_int, C.c_int, C.c_int, P(SSS_MAT), dp, C.c_int]),
            "ora_cf_jacobi": (None, [dp, P(SSS_MAT), dp, C.c_int, ip]),
            "ora_cf_jacobi_w": (None, [dp, P(SSS_MAT), dp, C.c_int, ip, C.c_double, C.c_int]),
            "ora_cf_twostage": (None, [dp, P(SSS_MAT), dp, C.c_int, ip, C.c_int]),
            "ora_smoother_pre": (None, [P(SSS_SMTR)]),
            "ora_smoother_post": (None, [P(SSS_SMTR)]),
            "ora_cg": (C.c_int, [P(SSS_KRYLOV), C.c_int]),
            "ora_gmres": (C.c_int, [P(SSS_KRYLOV), C.c_int]),
            "ora_coarest_solve": (None, [P(SSS_MAT), P(SSS_VEC), P(SSS_VEC), C.c_double, P(ORA_OPTS)]),
            "ora_cycle": (None, [P(SSS_AMG), P(ORA_OPTS)]),
            "ora_solve": (SSS_RTN, [P(SSS_AMG), P(SSS_VEC), P(SSS_VEC), P(ORA_OPTS), dp, dp, C.c_int]),
            "ora_coarse_seconds": (C.c_double, []),
            "ora_reset_timers": (None, []),
            "ora_interp_std": (None, [P(SSS_MAT), ip, P(SSS_MAT), P(SSS_IMAT), C.c_double]),
        }
        for name, (res, args) in sigs.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _ora = lib
    return _ora


def opts(**kw) -> ORA_OPTS:
    o = ORA_OPTS()
    load().ora_opts_default(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def load_ref():
    """The reference's own pure-C units, or None when they were not built (no reference tree)."""
    global _ref
    if _ref is None and REF_PATH.exists():
        lib = C.CDLL(str(REF_PATH), mode=os.RTLD_LAZY | os.RTLD_LOCAL)
        P = C.POINTER
        dp, ip = P(C.c_double), P(C.c_int)
        sigs = {
            "SSS_blas_mv_amxpy": (None, [C.c_double, P(SSS_MAT), P(SSS_VEC), P(SSS_VEC)]),
            "SSS_blas_mv_mxy": (None, [P(SSS_MAT), P(SSS_VEC), P(SSS_VEC)]),
            "SSS_amg_smoother_pre": (None, [P(SSS_SMTR)]),
            "SSS_amg_smoother_post": (None, [P(SSS_SMTR)]),
            "SSS_amg_coarsen": (C.c_int, [P(SSS_MAT), P(SSS_IVEC), P(SSS_MAT), P(SSS_IMAT), C.c_void_p]),
            "SSS_mat_trans": (SSS_MAT, [P(SSS_MAT)]),
            "SSS_blas_mat_rap": (SSS_MAT, [P(SSS_MAT), P(SSS_MAT), P(SSS_MAT)]),
            "SSS_mat_read": (None, [C.c_char_p, P(SSS_MAT)]),
            "SSS_amg_pars_init": (None, [C.c_void_p]),
            "SSS_blas_array_dot": (C.c_double, [C.c_int, dp, dp]),
            "SSS_blas_array_norm2": (C.c_double, [C.c_int, dp]),
            "SSS_ivec_create": (SSS_IVEC, [C.c_int]),
            # Solve/SSS_SOLVE.c, its SSS_amg_cycle resolved to ora_cycle (ref_cycle_glue.c)
            "SSS_amg_solve": (SSS_RTN, [P(SSS_AMG), P(SSS_VEC), P(SSS_VEC)]),
        }
        for name, (res, args) in sigs.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _ref = lib
    return _ref
