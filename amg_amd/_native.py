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
LIB_PATH = ROOT / "amg_amd" / "lib" / "libsss_amg.so"
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
                ("inner", C.c_int), ("inner_from", C.c_int), ("relabel", C.c_int)]


class SSS_HIP_LEVEL_INFO(C.Structure):
    _fields_ = [("rows", C.c_int), ("nnz", C.c_int), ("nnz_p", C.c_int), ("dag_f", C.c_int),
                ("dag_c", C.c_int), ("smoother_kind", C.c_int)]


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
    "sss_hip_opts_default", "sss_hip_device_count", "sss_hip_hier_create", "sss_hip_hier_destroy",
    "sss_hip_upload_vec", "sss_hip_download_vec", "sss_hip_cycle", "sss_hip_residual_norm",
    "sss_hip_coarse_solve", "sss_hip_smooth", "sss_hip_sync", "sss_hip_level_info_get", "sss_hip_num_levels",
    "sss_hip_spmv_plan_create", "sss_hip_spmv_plan_destroy", "sss_hip_spmv", "sss_hip_host_spmv",
    "sss_hip_host_smooth", "sss_hip_host_coarse_solve", "sss_hip_time_level0_spmv", "sss_hip_time_iterations",
    "sss_gen_stencil",
]

_lib = None


def _declare(lib):
    P = C.POINTER
    sig = {
        "SSS_amg_pars_init": (None, [P(SSS_AMG_PARS)]),
        "SSS_amg_pars_print": (None, [P(SSS_AMG_PARS)]),
        "SSS_amg_setup": (None, [P(SSS_AMG), P(SSS_MAT), P(SSS_AMG_PARS)]),
        "SSS_amg_data_destroy": (None, [P(SSS_AMG)]),
        "SSS_amg_solve": (SSS_RTN, [P(SSS_AMG), P(SSS_VEC), P(SSS_VEC)]),
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
        "sss_hip_hier_create": (C.c_void_p, [P(SSS_AMG), P(SSS_HIP_OPTS)]),
        "sss_hip_hier_destroy": (None, [C.c_void_p]),
        "sss_hip_upload_vec": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _dbl_p, C.c_int]),
        "sss_hip_download_vec": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _dbl_p, C.c_int]),
        "sss_hip_cycle": (C.c_int, [C.c_void_p]),
        "sss_hip_residual_norm": (C.c_int, [C.c_void_p, _dbl_p]),
        "sss_hip_coarse_solve": (C.c_int, [C.c_void_p]),
        "sss_hip_smooth": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
        "sss_hip_sync": (C.c_int, [C.c_void_p]),
        "sss_hip_level_info_get": (C.c_int, [C.c_void_p, C.c_int, P(SSS_HIP_LEVEL_INFO)]),
        "sss_hip_num_levels": (C.c_int, [C.c_void_p]),
        "sss_hip_host_spmv": (C.c_int, [C.c_int, C.c_double, P(SSS_MAT), _dbl_p, _dbl_p, _dbl_p, C.c_int]),
        "sss_hip_host_smooth": (C.c_int, [P(SSS_SMTR), C.c_int]),
        "sss_hip_host_coarse_solve": (C.c_int, [P(SSS_MAT), P(SSS_VEC), P(SSS_VEC), C.c_double, C.c_int,
                                                C.c_int]),
        "sss_hip_time_level0_spmv": (C.c_int, [C.c_void_p, C.c_int, _dbl_p]),
        "sss_hip_time_iterations": (C.c_int, [C.c_void_p, C.c_int, _dbl_p, _dbl_p]),
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
    """An SSS_AMG built by the (host C, reference-semantics) setup; owns it."""

    def __init__(self, A: SSS_MAT, pars: SSS_AMG_PARS | None = None):
        self.pars = pars if pars is not None else default_pars()
        self.mg = SSS_AMG()
        lib().SSS_amg_setup(C.byref(self.mg), C.byref(A), C.byref(self.pars))

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

    def __init__(self, H: Hierarchy, smoother: str = "exact", coarse: str = "krylov", row_cap: int = 0,
                 device: int = -1, verbose: int = 0, relabel: int | None = None, graph: int | None = None,
                 inner: int | None = None, inner_from: int | None = None):
        o = SSS_HIP_OPTS()
        lib().sss_hip_opts_default(C.byref(o))
        o.smoother, o.coarse, o.row_cap, o.device, o.verbose = SMOOTH[smoother], COARSE[coarse], row_cap, device, verbose
        if relabel is not None:
            o.relabel = relabel
        if graph is not None:
            o.use_graph = graph
        if inner is not None:
            o.inner = inner
        if inner_from is not None:
            o.inner_from = inner_from
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


def device_count() -> int:
    return lib().sss_hip_device_count()
