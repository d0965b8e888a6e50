"""ctypes mirror of the drop-in C ABI (include/sss_amg.h) and the device engine (include/sss_hip.h).

This is the host-side binding a Python caller (tests, bench.py) uses; the product itself is the
C-ABI library ``amg_amd/lib/libsss_amg.so``.  Struct layouts follow SSS_main.h:95-251 of the
reference exactly (sizes are asserted in tests/test_abi.py against SURVEY.md §8b).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
# SSS_AMG_LIB: an alternative build of the same library (A/B runs against a previous commit's
# build, tools/gpu/ab_env.sh)
LIB_PATH = Path(os.environ["SSS_AMG_LIB"]) if os.environ.get("SSS_AMG_LIB") else ROOT / "amg_amd" / "lib" / "libsss_amg.so"
BIN_PATH = ROOT / "amg_amd" / "bin" / "amg"

_dbl_p = C.POINTER(C.c_double)
_int_p = C.POINTER(C.c_int)


class SSS_MAT(C.Structure):
    _fields_ = [("num_rows", C.c_int), ("num_cols", C.c_int), ("num_nnzs", C.c_int),
                ("row_ptr", _int_p), ("col_idx", _int_p), ("val", _dbl_p)]


class SSS_IMAT(C.Structure):
    _fields_ = [("num_rows", C.c_int), ("num_cols", C.c_int), ("num_nnzs", C.c_int),
                ("row_ptr", _int_p), ("col_idx", _int_p), ("val", _int_p)]


class SSS_VEC(C.Structure):
    _fields_ = [("n", C.c_int), ("d", _dbl_p)]


class SSS_IVEC(C.Structure):
    _fields_ = [("n", C.c_int), ("d", _int_p)]


class SSS_RTN(C.Structure):
    _fields_ = [("ares", C.c_double), ("rres", C.c_double), ("nits", C.c_int)]


class SSS_AMG_PARS(C.Structure):
    _fields_ = [("cycle_type", C.c_int), ("tol", C.c_double), ("ctol", C.c_double), ("max_it", C.c_int),
                ("cs_type", C.c_int), ("max_levels", C.c_int), ("coarse_dof", C.c_int), ("smoother", C.c_int),
                ("relax", C.c_double), ("cf_order", C.c_int), ("pre_iter", C.c_int), ("post_iter", C.c_int),
                ("poly_deg", C.c_int), ("interp_type", C.c_int), ("strong_threshold", C.c_double),
                ("max_row_sum", C.c_double), ("trunc_threshold", C.c_double)]


class SSS_AMG_COMP(C.Structure):
    _fields_ = [("A", SSS_MAT), ("R", SSS_MAT), ("P", SSS_MAT), ("b", SSS_VEC), ("x", SSS_VEC),
                ("cfmark", SSS_IVEC), ("wp", SSS_VEC)]


class SSS_AMG(C.Structure):
    _fields_ = [("num_levels", C.c_int), ("cg", C.POINTER(SSS_AMG_COMP)), ("pars", SSS_AMG_PARS),
                ("rtn", SSS_RTN)]


class SSS_SMTR(C.Structure):
    _fields_ = [("smoother", C.c_int), ("A", C.POINTER(SSS_MAT)), ("b", C.POINTER(SSS_VEC)),
                ("x", C.POINTER(SSS_VEC)), ("relax", C.c_double), ("nsweeps", C.c_int), ("istart", C.c_int),
                ("iend", C.c_int), ("istep", C.c_int), ("ndeg", C.c_int), ("cf_order", C.c_int),
                ("ordering", _int_p)]


class SSS_KRYLOV(C.Structure):
    _fields_ = [("tol", C.c_double), ("A", C.POINTER(SSS_MAT)), ("b", C.POINTER(SSS_VEC)),
                ("u", C.POINTER(SSS_VEC)), ("restart", C.c_int), ("matrix", C.c_int), ("stop_type", C.c_int)]


class SSS_HIP_OPTS(C.Structure):
    _fields_ = [("device", C.c_int), ("smoother", C.c_int), ("coarse", C.c_int), ("row_cap", C.c_int),
                ("use_graph", C.c_int), ("verbose", C.c_int),
                ("inner", C.c_int), ("inner_from", C.c_int), ("relabel", C.c_int),
                ("sorted_tiles", C.c_int), ("sum_order", C.c_int), ("inner_long", C.c_int), ("formats", C.c_int)]

FORMATS = {"auto": -1, "full": 0, "lean": 1}


class SSS_HIP_LEVEL_INFO(C.Structure):
    _fields_ = [("rows", C.c_int), ("nnz", C.c_int), ("nnz_p", C.c_int), ("dag_f", C.c_int),
                ("dag_c", C.c_int), ("smoother_kind", C.c_int), ("gs_engine_f", C.c_int), ("gs_engine_c", C.c_int),
                ("gs_stall", C.c_int), ("a_format", C.c_int), ("a_stream_bytes", C.c_longlong),
                ("inner", C.c_int), ("r_format", C.c_int), ("p_format", C.c_int), ("pad_", C.c_int)]


SMOOTH = {"exact": 0, "hybrid": 1, "jacobi": 2}
COARSE = {"krylov": 0, "direct": 1}
VEC = {"b": 0, "x": 1, "wp": 2}
SPMV = {"mxy": 0, "amxpy": 1, "resid": 2, "acc": 3}

#: every symbol include/sss_amg.h and include/sss_hip.h declare (export check in tests)
ABI_SYMBOLS = [
    "SSS_amg_solve", "SSS_amg_cycle", "SSS_amg_coarest_solve", "SSS_amg_smoother_pre", "SSS_amg_smoother_post",
    "SSS_blas_mv_amxpy", "SSS_blas_mv_mxy", "SSS_solver_amg", "SSS_get_time", "SSS_free", "SSS_blas_vec_norm2",
    "SSS_print_itinfo", "SSS_exit_on_errcode", "SSS_blas_array_norm2", "SSS_blas_array_dot", "SSS_blas_array_axpy",
    "SSS_blas_array_norminf", "SSS_blas_array_set", "SSS_blas_array_axpby", "SSS_blas_array_ax", "SSS_vec_create",
    "SSS_vec_set_value", "SSS_mat_destroy", "SSS_vec_destroy", "SSS_calloc", "SSS_amg_data_create",
    "SSS_ivec_create", "SSS_mat_struct_create", "SSS_vec_cp", "SSS_iarray_cp", "SSS_blas_array_cp", "SSS_mat_cp",
    "SSS_mat_get_diag", "SSS_ivec_destroy", "SSS_amg_data_destroy", "SSS_imat_trans", "SSS_iarray_set",
    "SSS_imat_destroy", "SSS_mat_trans", "SSS_blas_mat_rap", "SSS_realloc", "SSS_amg_complexity_print",
    "SSS_amg_setup", "SSS_amg_coarsen", "SSS_amg_interp", "SSS_amg_interp_trunc", "interp_DIR", "SSS_mat_read",
    "SSS_amg_pars_init", "SSS_amg_pars_print", "mmio_info", "mmio_data",
    "sss_hip_opts_default", "sss_hip_device_count", "sss_hip_mem_info", "sss_hip_hier_create", "sss_hip_hier_destroy",
    "sss_hip_setup_create", "sss_amg_setup_hooked", "sss_hip_rap",
    "sss_hip_upload_vec", "sss_hip_download_vec", "sss_hip_cycle", "sss_hip_residual_norm", "sss_hip_pcg",
    "SSS_amg_save", "SSS_amg_load",
    "sss_hip_coarse_solve", "sss_hip_smooth", "sss_hip_sync", "sss_hip_level_info_get", "sss_hip_num_levels", "sss_hip_tail_from",
    "sss_hip_cycle_launches", "sss_hip_cycle_bytes",
    "sss_hip_spmv_plan_create", "sss_hip_spmv_plan_destroy", "sss_hip_spmv", "sss_hip_host_spmv",
    "sss_hip_host_smooth", "sss_hip_host_coarse_solve", "sss_hip_host_cache_clear", "sss_hip_time_level0_spmv", "sss_hip_time_iterations",
    "sss_hip_time_level0_spmv_csr", "sss_hip_time_levels", "sss_hip_dist_time_tail_levels",
    "sss_gen_stencil",
    "sss_hip_rccl_unique_id", "sss_hip_comm_rccl", "sss_hip_comm_host", "sss_hip_comm_timing", "sss_hip_comm_destroy",
    "sss_hip_dist_create", "sss_hip_dist_destroy", "sss_hip_dist_info", "sss_hip_dist_level_flags",
    "sss_hip_dist_upload_vec",
    "sss_hip_dist_download_vec", "sss_hip_dist_cycle", "sss_hip_dist_residual_norm", "sss_hip_dist_sync",
    "sss_hip_dist_time_level0_spmv", "sss_hip_dist_time_levels", "sss_hip_dist_halo_stats",
    "sss_part_plan_create", "sss_part_plan_destroy", "sss_part_save", "sss_part_plan_load",
    "sss_hip_dist_create_from_files", "sss_hip_dist_level_size", "sss_part_plan_nagg", "sss_part_plan_level",
    "sss_part_plan_matrix", "sss_part_plan_ids", "sss_part_plan_halo",
]

_ip, _dp = C.POINTER(C.c_int), C.POINTER(C.c_double)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, _ip, _ip, _dp, C.c_int, _ip, _ip, _dp)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, _dp, C.c_int)
ALLGATHERV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, _dp, C.c_int, _dp, _ip, _ip)


# sss_hip_level_info::a_format & 3 -> storage format of a level operator
A_FORMATS = {0: "CSR (12 B/entry)", 1: "column-sorted tiles (12 B/entry)", 2: "dictionary tiles (4 B/entry)",
             3: "value-dictionary sorted tiles (5 B/entry)"}


def a_format_name(code: int) -> str:
    if code & 64:
        return "dictionary ELL (1 B/entry, padded rows)"
    if code & 128:
        return "column ELL (4 B/entry, padded rows)"
    return A_FORMATS.get(code & 3, A_FORMATS[0])


class SSS_HIP_HOST_TRANSPORT(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("exchange", EXCHANGE_FN), ("allreduce_sum", ALLREDUCE_FN),
                ("allgatherv", ALLGATHERV_FN)]

_lib = None


def _declare(lib):
    P = C.POINTER
    sig = {
        "SSS_amg_pars_init": (None, [P(SSS_AMG_PARS)]),
        "SSS_amg_pars_print": (None, [P(SSS_AMG_PARS)]),
        "SSS_amg_setup": (None, [P(SSS_AMG), P(SSS_MAT), P(SSS_AMG_PARS)]),
        "SSS_amg_data_destroy": (None, [P(SSS_AMG)]),
        "SSS_amg_solve": (SSS_RTN, [P(SSS_AMG), P(SSS_VEC), P(SSS_VEC)]),
        "SSS_print_itinfo": (None, [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double]),
        "SSS_amg_cycle": (None, [P(SSS_AMG)]),
        "SSS_solver_amg": (SSS_RTN, [P(SSS_MAT), P(SSS_VEC), P(SSS_VEC), P(SSS_AMG_PARS)]),
        "SSS_mat_read": (None, [C.c_char_p, P(SSS_MAT)]),
        "SSS_mat_destroy": (None, [P(SSS_MAT)]),
        "SSS_mat_trans": (SSS_MAT, [P(SSS_MAT)]),
        "SSS_blas_mat_rap": (SSS_MAT, [P(SSS_MAT), P(SSS_MAT), P(SSS_MAT)]),
        "SSS_amg_coarsen": (C.c_int, [P(SSS_MAT), P(SSS_IVEC), P(SSS_MAT), P(SSS_IMAT), P(SSS_AMG_PARS)]),
        "SSS_amg_interp": (None, [P(SSS_MAT), P(SSS_IVEC), P(SSS_MAT), P(SSS_IMAT), P(SSS_AMG_PARS)]),
        "SSS_ivec_create": (SSS_IVEC, [C.c_int]),
        "SSS_blas_mv_amxpy": (None, [C.c_double, P(SSS_MAT), P(SSS_VEC), P(SSS_VEC)]),
        "SSS_blas_mv_mxy": (None, [P(SSS_MAT), P(SSS_VEC), P(SSS_VEC)]),
        "mmio_info": (C.c_int, [_int_p, _int_p, _int_p, _int_p, C.c_char_p]),
        "mmio_data": (C.c_int, [_int_p, _int_p, _dbl_p, C.c_char_p]),
        "sss_gen_stencil": (C.c_int, [C.c_int] * 6 + [P(SSS_MAT)]),
        "sss_hip_opts_default": (None, [P(SSS_HIP_OPTS)]),
        "sss_hip_device_count": (C.c_int, []),
        "sss_hip_mem_info": (C.c_int, [P(C.c_size_t), P(C.c_size_t)]),
        "sss_hip_hier_create": (C.c_void_p, [P(SSS_AMG), P(SSS_HIP_OPTS)]),
        "sss_hip_setup_create": (C.c_void_p, [P(SSS_AMG), P(SSS_MAT), P(SSS_AMG_PARS), P(SSS_HIP_OPTS),
                                              P(C.c_double)]),
        "sss_hip_hier_destroy": (None, [C.c_void_p]),
        "sss_hip_rap": (C.c_int, [P(SSS_MAT), P(SSS_MAT), P(SSS_MAT), P(SSS_MAT)]),
        "sss_hip_upload_vec": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _dbl_p, C.c_int]),
        "sss_hip_download_vec": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _dbl_p, C.c_int]),
        "sss_hip_cycle": (C.c_int, [C.c_void_p]),
        "sss_hip_residual_norm": (C.c_int, [C.c_void_p, _dbl_p]),
        "sss_hip_pcg": (C.c_int, [C.c_void_p, C.c_double, C.c_int, P(C.c_int), _dbl_p, _dbl_p, C.c_int]),
        "SSS_amg_save": (C.c_int, [P(SSS_AMG), C.c_char_p]),
        "SSS_amg_load": (C.c_int, [P(SSS_AMG), C.c_char_p]),
        "sss_hip_coarse_solve": (C.c_int, [C.c_void_p]),
        "sss_hip_smooth": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
        "sss_hip_sync": (C.c_int, [C.c_void_p]),
        "sss_hip_level_info_get": (C.c_int, [C.c_void_p, C.c_int, P(SSS_HIP_LEVEL_INFO)]),
        "sss_hip_num_levels": (C.c_int, [C.c_void_p]),
        "sss_hip_tail_from": (C.c_int, [C.c_void_p]),
        "sss_hip_cycle_launches": (C.c_int, [C.c_void_p]),
        "sss_hip_cycle_bytes": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.c_int]),
        "sss_hip_host_spmv": (C.c_int, [C.c_int, C.c_double, P(SSS_MAT), _dbl_p, _dbl_p, _dbl_p, C.c_int]),
        "sss_hip_host_smooth": (C.c_int, [P(SSS_SMTR), C.c_int]),
        "sss_hip_host_coarse_solve": (C.c_int, [P(SSS_MAT), P(SSS_VEC), P(SSS_VEC), C.c_double, C.c_int,
                                                C.c_int]),
        "sss_hip_time_level0_spmv": (C.c_int, [C.c_void_p, C.c_int, _dbl_p]),
        "sss_hip_time_level0_spmv_csr": (C.c_int, [C.c_void_p, C.c_int, _dbl_p]),
        "sss_hip_time_levels": (C.c_int, [C.c_void_p, C.c_int, _dbl_p, C.c_int]),
        "sss_hip_dist_time_tail_levels": (C.c_int, [C.c_void_p, C.c_int, _dbl_p, C.c_int]),
        "sss_hip_time_iterations": (C.c_int, [C.c_void_p, C.c_int, _dbl_p, _dbl_p]),
        "sss_hip_rccl_unique_id": (C.c_int, [C.c_char_p]),
        "sss_hip_comm_rccl": (C.c_void_p, [C.c_int, C.c_int, C.c_char_p, C.c_int]),
        "sss_hip_comm_host": (C.c_void_p, [C.c_int, C.c_int, P(SSS_HIP_HOST_TRANSPORT)]),
        "sss_hip_comm_timing": (C.c_void_p, [C.c_int, C.c_int]),
        "sss_hip_comm_destroy": (None, [C.c_void_p]),
        "sss_hip_dist_create": (C.c_void_p, [P(SSS_AMG), P(SSS_HIP_OPTS), C.c_void_p, C.c_int]),
        "sss_hip_dist_destroy": (None, [C.c_void_p]),
        "sss_hip_dist_info": (C.c_int, [C.c_void_p, _int_p, _int_p, _int_p, _int_p]),
        "sss_hip_dist_level_size": (C.c_int, [C.c_void_p, C.c_int, _int_p, _int_p, P(C.c_longlong)]),
        "sss_hip_dist_level_flags": (C.c_int, [C.c_void_p, C.c_int]),
        "sss_hip_dist_upload_vec": (C.c_int, [C.c_void_p, C.c_int, _dbl_p, C.c_int]),
        "sss_hip_dist_download_vec": (C.c_int, [C.c_void_p, C.c_int, _dbl_p, C.c_int]),
        "sss_hip_dist_cycle": (C.c_int, [C.c_void_p]),
        "sss_hip_dist_residual_norm": (C.c_int, [C.c_void_p, _dbl_p]),
        "sss_hip_dist_sync": (C.c_int, [C.c_void_p]),
        "sss_hip_dist_time_level0_spmv": (C.c_int, [C.c_void_p, C.c_int, _dbl_p]),
        "sss_hip_dist_time_levels": (C.c_int, [C.c_void_p, C.c_int, _dbl_p, _dbl_p, C.c_int]),
        "sss_hip_dist_halo_stats": (C.c_int, [C.c_void_p, P(C.c_longlong), P(C.c_longlong), C.c_int, C.c_int,
                                              _int_p, _int_p, _int_p]),
        "sss_part_plan_create": (C.c_void_p, [P(SSS_AMG), C.c_int, C.c_int, C.c_int]),
        "sss_part_save": (C.c_int, [P(SSS_AMG), C.c_int, C.c_int, C.c_char_p]),
        "sss_part_plan_load": (C.c_void_p, [C.c_char_p]),
        "sss_hip_dist_create_from_files": (C.c_void_p, [C.c_char_p, P(SSS_HIP_OPTS), C.c_void_p]),
        "sss_part_plan_destroy": (None, [C.c_void_p]),
        "sss_part_plan_nagg": (C.c_int, [C.c_void_p]),
        "sss_part_plan_level": (C.c_int, [C.c_void_p, C.c_int, _int_p, _int_p, _int_p, _int_p]),
        "sss_part_plan_matrix": (C.c_int, [C.c_void_p, C.c_int, C.c_int, P(SSS_MAT)]),
        "sss_part_plan_ids": (C.c_int, [C.c_void_p, C.c_int, P(_int_p), P(_int_p)]),
        "sss_part_plan_halo": (C.c_int, [C.c_void_p, C.c_int, _int_p, P(_int_p), P(_int_p), P(_int_p), _int_p,
                                         P(_int_p), P(_int_p)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def lib():
    """Load libsss_amg.so (built by `make` / __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} is missing: run `make` (or __graft_entry__.build())")
        _lib = _declare(C.CDLL(str(LIB_PATH)))
    return _lib


def dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_dbl_p)


def iptr(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_int_p)


def csr_arrays(M: SSS_MAT, copy: bool = True):
    """(row_ptr, col_idx, val) numpy views (copies by default) of a C-owned SSS_MAT."""
    n, nnz = M.num_rows, M.num_nnzs
    rp = np.ctypeslib.as_array(M.row_ptr, shape=(n + 1,))
    ci = np.ctypeslib.as_array(M.col_idx, shape=(nnz,)) if nnz else np.zeros(0, np.int32)
    v = np.ctypeslib.as_array(M.val, shape=(nnz,)) if nnz else np.zeros(0, np.float64)
    return (rp.copy(), ci.copy(), v.copy()) if copy else (rp, ci, v)


class NumpyCSR:
    """Keeps numpy buffers alive behind an SSS_MAT view (host memory owned by Python)."""

    def __init__(self, rp, ci, v, ncols=None):
        self.rp = np.ascontiguousarray(rp, dtype=np.int32)
        self.ci = np.ascontiguousarray(ci, dtype=np.int32)
        self.v = np.ascontiguousarray(v, dtype=np.float64)
        n = len(self.rp) - 1
        self.mat = SSS_MAT(n, n if ncols is None else ncols, len(self.v), iptr(self.rp), iptr(self.ci),
                           dptr(self.v))


def default_pars() -> SSS_AMG_PARS:
    p = SSS_AMG_PARS()
    lib().SSS_amg_pars_init(C.byref(p))
    return p


def generate(kind: int, n: int, nz: int | None = None, z0: int = 0, z1: int | None = None) -> SSS_MAT:
    """7-point or 27-point (anisotropic) stencil on an n*n*nz grid, rows of planes [z0, z1)."""
    nz = n if nz is None else nz
    z1 = nz if z1 is None else z1
    A = SSS_MAT()
    rc = lib().sss_gen_stencil(kind, n, n, nz, z0, z1, C.byref(A))
    if rc != 0:
        raise RuntimeError(f"sss_gen_stencil failed ({rc})")
    return A


def read_mtx(path: str | os.PathLike) -> SSS_MAT:
    A = SSS_MAT()
    lib().SSS_mat_read(str(path).encode(), C.byref(A))
    return A


class Hierarchy:
    """An SSS_AMG built by the (host C, reference-semantics) setup -- or read back from a file
    SSS_amg_save wrote (Hierarchy.load) -- owns it."""

    def __init__(self, A: SSS_MAT | None, pars: SSS_AMG_PARS | None = None):
        self.pars = pars if pars is not None else default_pars()
        self.mg = SSS_AMG()
        if A is not None:
            lib().SSS_amg_setup(C.byref(self.mg), C.byref(A), C.byref(self.pars))

    def save(self, path) -> None:
        rc = lib().SSS_amg_save(C.byref(self.mg), str(path).encode())
        if rc != 0:
            raise OSError(f"SSS_amg_save({path}) failed ({rc})")

    @classmethod
    def load(cls, path) -> "Hierarchy":
        H = cls(None)
        rc = lib().SSS_amg_load(C.byref(H.mg), str(path).encode())
        if rc != 0:
            raise OSError(f"SSS_amg_load({path}) failed ({rc})")
        H.pars = H.mg.pars
        return H

    @property
    def num_levels(self) -> int:
        return self.mg.num_levels

    def level(self, l: int) -> SSS_AMG_COMP:
        return self.mg.cg[l]

    def close(self):
        if self.mg.cg:
            lib().SSS_amg_data_destroy(C.byref(self.mg))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceHierarchy:
    """HBM mirror of a Hierarchy (sss_hip_hier_create)."""

    def __init__(self, H: Hierarchy | None, smoother: str = "exact", coarse: str = "krylov", row_cap: int = 0,
                 device: int = -1, verbose: int = 0, relabel: int | None = None, graph: int | None = None,
                 inner: int | None = None, inner_from: int | None = None, sorted_tiles: int | None = None,
                 sum_order: int | None = None, setup_from: SSS_MAT | None = None, inner_long: int | None = None,
                 formats: str | None = None):
        """setup_from: build the Hierarchy from this operator here, with the levels uploaded while
        the setup is still running (sss_hip_setup_create); H must then be None and self.H is the
        new Hierarchy.  self.times = (setup s, mirror s after the setup, of which waiting)."""
        o = SSS_HIP_OPTS()
        lib().sss_hip_opts_default(C.byref(o))
        o.smoother, o.coarse, o.row_cap, o.device, o.verbose = SMOOTH[smoother], COARSE[coarse], row_cap, device, verbose
        if sorted_tiles is not None:
            o.sorted_tiles = sorted_tiles
        if sum_order is not None:
            o.sum_order = sum_order
        if relabel is not None:
            o.relabel = relabel
        if graph is not None:
            o.use_graph = graph
        if inner is not None:
            o.inner = inner
        if inner_from is not None:
            o.inner_from = inner_from
        if inner_long is not None:
            o.inner_long = inner_long
        if formats is not None:
            o.formats = FORMATS[formats]
        if setup_from is not None:
            if H is not None:
                raise ValueError("setup_from builds its own Hierarchy: pass H=None")
            H = Hierarchy(None)
            t = (C.c_double * 3)()
            self.H = H
            self.h = lib().sss_hip_setup_create(C.byref(H.mg), C.byref(setup_from), C.byref(H.pars), C.byref(o), t)
            self.times = tuple(t)
            if not self.h:
                raise RuntimeError("sss_hip_setup_create failed (no HIP device or out of memory)")
            return
        self.H = H
        self.h = lib().sss_hip_hier_create(C.byref(H.mg), C.byref(o))
        if not self.h:
            raise RuntimeError("sss_hip_hier_create failed (no HIP device or out of memory)")

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc})")

    def upload(self, level: int, which: str, a: np.ndarray):
        a = np.ascontiguousarray(a, dtype=np.float64)
        self._check(lib().sss_hip_upload_vec(self.h, level, VEC[which], dptr(a), len(a)), "upload")

    def download(self, level: int, which: str, n: int | None = None) -> np.ndarray:
        n = self.H.level(level).A.num_rows if n is None else n
        out = np.empty(n, np.float64)
        self._check(lib().sss_hip_download_vec(self.h, level, VEC[which], dptr(out), n), "download")
        return out

    def cycle(self):
        self._check(lib().sss_hip_cycle(self.h), "cycle")

    def residual_norm(self) -> float:
        out = C.c_double()
        self._check(lib().sss_hip_residual_norm(self.h, C.byref(out)), "residual_norm")
        return out.value

    def pcg(self, tol: float, maxit: int = 100):
        """AMG-preconditioned CG on level 0 (b, x uploaded as for cycle()); returns (iterations,
        relative residual history)."""
        hist = np.zeros(max(maxit, 1))
        its, rel = C.c_int(), C.c_double()
        self._check(lib().sss_hip_pcg(self.h, tol, maxit, C.byref(its), C.byref(rel), dptr(hist), len(hist)), "pcg")
        return its.value, hist[: its.value].copy()

    def smooth(self, level: int, post: bool):
        self._check(lib().sss_hip_smooth(self.h, level, int(post)), "smooth")

    def coarse_solve(self):
        self._check(lib().sss_hip_coarse_solve(self.h), "coarse_solve")

    def sync(self):
        self._check(lib().sss_hip_sync(self.h), "sync")

    def level_info(self, level: int) -> SSS_HIP_LEVEL_INFO:
        info = SSS_HIP_LEVEL_INFO()
        self._check(lib().sss_hip_level_info_get(self.h, level, C.byref(info)), "level_info")
        return info

    def time_level0_spmv(self, reps: int) -> float:
        ms = C.c_double()
        self._check(lib().sss_hip_time_level0_spmv(self.h, reps, C.byref(ms)), "time_level0_spmv")
        return ms.value

    def cycle_bytes(self) -> dict:
        """Stored-format bytes of one outer iteration (sss_hip_cycle_bytes): per level, the outer
        residual + norm, the coarsest solve, and their total."""
        nl = lib().sss_hip_num_levels(self.h)
        buf = (C.c_double * (nl + 2))()
        self._check(lib().sss_hip_cycle_bytes(self.h, buf, nl + 2), "cycle_bytes")
        v = list(buf)
        return {"levels": v[:nl], "outer": v[nl], "coarse": v[nl + 1], "total": sum(v)}

    def time_level0_spmv_csr(self, reps: int) -> float:
        """the same residual SpMV from A_0's plain CSR arrays (the metric's fine-level CSR SpMV)"""
        ms = C.c_double()
        self._check(lib().sss_hip_time_level0_spmv_csr(self.h, reps, C.byref(ms)), "time_level0_spmv_csr")
        return ms.value

    def time_levels(self, reps: int) -> list:
        """ms per level of an eager cycle (sss_hip_time_levels); advances the iterate"""
        lv = (C.c_double * self.H.num_levels)() if self.H is not None else (C.c_double * 32)()
        self._check(lib().sss_hip_time_levels(self.h, reps, lv, len(lv)), "time_levels")
        return list(lv)

    def time_iterations(self, reps: int):
        ms, ares = C.c_double(), C.c_double()
        self._check(lib().sss_hip_time_iterations(self.h, reps, C.byref(ms), C.byref(ares)), "time_iterations")
        return ms.value, ares.value

    def close(self):
        if self.h:
            lib().sss_hip_hier_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def hbm_used_bytes() -> int:
    """HBM in use on the current device (total - free, hipMemGetInfo): this process's mirrors plus
    the runtime's own allocations."""
    f, t = C.c_size_t(), C.c_size_t()
    if lib().sss_hip_mem_info(C.byref(f), C.byref(t)) != 0:
        raise RuntimeError("sss_hip_mem_info failed")
    return t.value - f.value


def device_count() -> int:
    return lib().sss_hip_device_count()


# ---------------------------------------------------------------- row-partitioned multi-GPU
def part_save(H: "Hierarchy", nranks: int, prefix, agg_rows: int = 0) -> None:
    """Partition set of H for nranks ranks (sss_part_save): prefix.r<rank> files + prefix.tail."""
    rc = lib().sss_part_save(C.byref(H.mg), nranks, agg_rows, str(prefix).encode())
    if rc != 0:
        raise OSError(f"sss_part_save({prefix}) failed ({rc})")


class PartPlan:
    """Host-only view of one rank's partition of a hierarchy (sss_part_plan_*), built from the
    global hierarchy, or read back from its partition file (PartPlan.load)."""

    def __init__(self, H: "Hierarchy | None", nranks: int = 1, rank: int = 0, agg_rows: int = 0):
        self.H = H
        self.p = None
        if H is not None:
            self.p = lib().sss_part_plan_create(C.byref(H.mg), nranks, rank, agg_rows)
            if not self.p:
                raise RuntimeError("sss_part_plan_create failed")
            self.nagg = lib().sss_part_plan_nagg(self.p)

    @classmethod
    def load(cls, path) -> "PartPlan":
        pp = cls(None)
        pp.p = lib().sss_part_plan_load(str(path).encode())
        if not pp.p:
            raise OSError(f"sss_part_plan_load({path}) failed")
        pp.nagg = lib().sss_part_plan_nagg(pp.p)
        return pp

    def level(self, l: int):
        lo, hi, m, g = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        assert lib().sss_part_plan_level(self.p, l, C.byref(lo), C.byref(hi), C.byref(m), C.byref(g)) == 0
        return lo.value, hi.value, m.value, g.value

    def matrix(self, l: int, which: str) -> SSS_MAT:
        M = SSS_MAT()
        assert lib().sss_part_plan_matrix(self.p, l, {"A": 0, "P": 1, "R": 2}[which], C.byref(M)) == 0
        return M

    def ids(self, l: int):
        _, _, m, g = self.level(l)
        pp, gp = _int_p(), _int_p()
        assert lib().sss_part_plan_ids(self.p, l, C.byref(pp), C.byref(gp)) == 0
        perm = np.ctypeslib.as_array(pp, shape=(m,)).copy() if m else np.zeros(0, np.int32)
        ghosts = np.ctypeslib.as_array(gp, shape=(g,)).copy() if g else np.zeros(0, np.int32)
        return perm, ghosts

    def halo(self, l: int):
        ns, nr = C.c_int(), C.c_int()
        sd, sc, si, rs, rc = _int_p(), _int_p(), _int_p(), _int_p(), _int_p()
        assert lib().sss_part_plan_halo(self.p, l, C.byref(ns), C.byref(sd), C.byref(sc), C.byref(si), C.byref(nr),
                                        C.byref(rs), C.byref(rc)) == 0

        def arr(ptr, n):
            return np.ctypeslib.as_array(ptr, shape=(n,)).copy() if n else np.zeros(0, np.int32)

        scount = arr(sc, ns.value)
        return dict(sdst=arr(sd, ns.value), scount=scount, sidx=arr(si, int(scount.sum())),
                    rsrc=arr(rs, nr.value), rcount=arr(rc, nr.value))

    def close(self):
        if self.p:
            lib().sss_part_plan_destroy(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TorchHostTransport:
    """sss_hip_host_transport over torch.distributed (gloo): the test transport of the
    distributed engine (several ranks may then share one GPU, which RCCL refuses)."""

    def __init__(self):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist

        def exchange(ctx, ns, sdst, scount, sbuf, nr, rsrc, rcount, rbuf):
            try:
                reqs, off = [], 0
                sc = [scount[i] for i in range(ns)]
                tot = sum(sc)
                sb = np.ctypeslib.as_array(sbuf, shape=(max(tot, 1),))
                for i in range(ns):
                    t = torch.from_numpy(sb[off:off + sc[i]].copy())
                    reqs.append(dist.isend(t, sdst[i]))
                    off += sc[i]
                rc = [rcount[i] for i in range(nr)]
                outs = []
                for i in range(nr):
                    t = torch.empty(rc[i], dtype=torch.float64)
                    reqs.append(dist.irecv(t, rsrc[i]))
                    outs.append(t)
                for r in reqs:
                    r.wait()
                if nr:
                    rb = np.ctypeslib.as_array(rbuf, shape=(sum(rc),))
                    off = 0
                    for i in range(nr):
                        rb[off:off + rc[i]] = outs[i].numpy()
                        off += rc[i]
                return 0
            except Exception as e:  # pragma: no cover - reported through the C return code
                print("transport exchange failed:", e, flush=True)
                return 1

        def allreduce(ctx, v, n):
            a = np.ctypeslib.as_array(v, shape=(n,))
            t = torch.from_numpy(a.copy())
            dist.all_reduce(t)
            a[:] = t.numpy()
            return 0

        def allgatherv(ctx, mine, count, out, counts, displs):
            W = dist.get_world_size()
            cnt = [counts[q] for q in range(W)]
            mx = max(max(cnt), 1)
            buf = torch.zeros(mx, dtype=torch.float64)
            if count:
                buf[:count] = torch.from_numpy(np.ctypeslib.as_array(mine, shape=(count,)).copy())
            parts = [torch.zeros(mx, dtype=torch.float64) for _ in range(W)]
            dist.all_gather(parts, buf)
            o = np.ctypeslib.as_array(out, shape=(sum(cnt),))
            for q in range(W):
                o[displs[q]:displs[q] + cnt[q]] = parts[q][:cnt[q]].numpy()
            return 0

        self._fns = (EXCHANGE_FN(exchange), ALLREDUCE_FN(allreduce), ALLGATHERV_FN(allgatherv))
        self.t = SSS_HIP_HOST_TRANSPORT(None, *self._fns)


class Comm:
    """sss_hip_comm: RCCL (one GPU per rank), the host transport (tests), or "timing": no transfer at all
    (the per-rank compute floor, tools/n8_floor.py; iterates meaningless)."""

    def __init__(self, nranks: int, rank: int, kind: str = "rccl", device: int = -1):
        self.kind = kind
        if kind == "rccl":
            import torch
            import torch.distributed as dist
            uid = C.create_string_buffer(128)
            ok = 1
            if rank == 0:
                ok = int(lib().sss_hip_rccl_unique_id(uid) == 0)
            # the id and rank 0's status together: a failed id fails every rank, none waits
            t = torch.frombuffer(bytearray(uid.raw[:128] + bytes([ok])), dtype=torch.uint8).clone()
            dist.broadcast(t, 0)
            raw = bytes(t.numpy().tobytes())
            if not raw[128]:
                raise RuntimeError("communicator (rccl) creation failed: no unique id on rank 0")
            uid = C.create_string_buffer(raw[:128], 128)
            self.c = lib().sss_hip_comm_rccl(nranks, rank, uid, device)
        elif kind == "timing":
            self.c = lib().sss_hip_comm_timing(nranks, rank)
        else:
            self.transport = TorchHostTransport()
            self.c = lib().sss_hip_comm_host(nranks, rank, C.byref(self.transport.t))
        if not self.c:
            raise RuntimeError(f"communicator ({kind}) creation failed")

    def close(self):
        if self.c:
            lib().sss_hip_comm_destroy(self.c)
            self.c = None


class DistHierarchy:
    """Row-partitioned device hierarchy (sss_hip_dist_*): this rank's rows of every level, built
    from the global hierarchy H, or (H None, parts = a partition-set prefix) from this rank's
    partition file and the tail file only."""

    def __init__(self, H: "Hierarchy | None", comm: Comm, smoother: str = "hybrid", coarse: str = "direct",
                 device: int = -1, agg_rows: int = 0, inner: int | None = None, inner_from: int | None = None,
                 sorted_tiles: int | None = None, sum_order: int | None = None, parts=None,
                 inner_long: int | None = None, formats: str | None = None):
        o = SSS_HIP_OPTS()
        lib().sss_hip_opts_default(C.byref(o))
        o.smoother, o.coarse, o.device = SMOOTH[smoother], COARSE[coarse], device
        if formats is not None:
            o.formats = FORMATS[formats]
        if sorted_tiles is not None:
            o.sorted_tiles = sorted_tiles
        if sum_order is not None:
            o.sum_order = sum_order
        if inner is not None:
            o.inner = inner
        if inner_from is not None:
            o.inner_from = inner_from
        if inner_long is not None:
            o.inner_long = inner_long
        self.H, self.comm = H, comm
        if H is None:
            self.d = lib().sss_hip_dist_create_from_files(str(parts).encode(), C.byref(o), comm.c)
        else:
            self.d = lib().sss_hip_dist_create(C.byref(H.mg), C.byref(o), comm.c, agg_rows)
        if not self.d:
            raise RuntimeError("sss_hip_dist_create failed")
        lo, hi, nagg, g = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        lib().sss_hip_dist_info(self.d, C.byref(lo), C.byref(hi), C.byref(nagg), C.byref(g))
        self.lo, self.hi, self.nagg, self.nghost0 = lo.value, hi.value, nagg.value, g.value

    def level_size(self, l: int):
        """(own rows, ghosts, nonzeros) of this rank's partitioned level l"""
        m, g, z = C.c_int(), C.c_int(), C.c_longlong()
        self._check(lib().sss_hip_dist_level_size(self.d, l, C.byref(m), C.byref(g), C.byref(z)), "level size")
        return m.value, g.value, z.value

    def level_flags(self, l: int) -> dict:
        """Exact eliminations in force on partitioned level l (agreed over the ranks)."""
        f = lib().sss_hip_dist_level_flags(self.d, l)
        if f < 0:
            raise ValueError(f"no partitioned level {l}")
        return {"zero_first": bool(f & 1), "fused_residual": bool(f & 2), "dead_prolong": bool(f & 4),
                "cycle_graph": bool(f & 8)}

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc})")

    def upload(self, which: str, own: np.ndarray):
        own = np.ascontiguousarray(own, dtype=np.float64)
        self._check(lib().sss_hip_dist_upload_vec(self.d, VEC[which], dptr(own), len(own)), "dist upload")

    def download(self, which: str) -> np.ndarray:
        out = np.empty(self.hi - self.lo, np.float64)
        self._check(lib().sss_hip_dist_download_vec(self.d, VEC[which], dptr(out), len(out)), "dist download")
        return out

    def cycle(self):
        self._check(lib().sss_hip_dist_cycle(self.d), "dist cycle")

    def residual_norm(self) -> float:
        r = C.c_double()
        self._check(lib().sss_hip_dist_residual_norm(self.d, C.byref(r)), "dist residual")
        return r.value

    def sync(self):
        self._check(lib().sss_hip_dist_sync(self.d), "dist sync")

    def time_level0_spmv(self, reps: int) -> float:
        ms = C.c_double()
        self._check(lib().sss_hip_dist_time_level0_spmv(self.d, reps, C.byref(ms)), "dist spmv timing")
        return ms.value

    def time_levels(self, reps: int):
        """(cycle ms as it runs, [per partitioned level ms of an eager cycle] + [replicated tail ms])"""
        cyc = C.c_double()
        lv = (C.c_double * (self.nagg + 1))()
        self._check(lib().sss_hip_dist_time_levels(self.d, reps, C.byref(cyc), lv, self.nagg + 1), "dist level timing")
        return cyc.value, list(lv)

    def time_tail_levels(self, reps: int) -> list:
        """ms per replicated level (global levels nagg, nagg + 1, ...) of the tail's own eager cycle"""
        lv = (C.c_double * 32)()
        self._check(lib().sss_hip_dist_time_tail_levels(self.d, reps, lv, 32), "tail level timing")
        return list(lv)

    def halo_stats(self, reset: bool = True) -> dict:
        calls = (C.c_longlong * self.nagg)()
        dbl = (C.c_longlong * self.nagg)()
        own, allr, tl = C.c_int(), C.c_int(), C.c_int()
        self._check(lib().sss_hip_dist_halo_stats(self.d, calls, dbl, self.nagg, int(reset), C.byref(own), C.byref(allr),
                                                  C.byref(tl)), "dist halo stats")
        return {"exchanges": list(calls), "doubles_sent": list(dbl), "gather_own": own.value, "gather_all": allr.value,
                "tail_levels": tl.value}

    def close(self):
        if self.d:
            lib().sss_hip_dist_destroy(self.d)
            self.d = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
