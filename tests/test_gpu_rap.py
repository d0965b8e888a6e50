"""GPU: the setup's Galerkin product on the device (sss_hip_rap, amg_amd/csrc/sss_rap.hip) against
the host product SSS_blas_mat_rap (amg_amd/host/sss_setup.c, itself bitwise the reference's
SSS_matvec.c:398-534 in tests/test_ref_units.py): same row pointers, same column order (diagonal
first, then first-discovery order), same values bit for bit -- on every level of stencil,
27-point, irregular and SuiteSparse hierarchies, with every device table size, with rows left to
the host fallback, and through whole setups (hierarchy digests equal with and without it)."""
from __future__ import annotations

import ctypes as C
import hashlib

import numpy as np
import pytest

import amg_amd as A
from amg_amd import workloads as W
from conftest import BUS_MTX, build_hierarchy, quiet_ctx

pytestmark = pytest.mark.gpu


def _mats(case):
    keep = None
    if case == "bus":
        M = A.read_mtx(BUS_MTX)
    elif case == "p7_32":
        M = A.generate(7, 32)
    elif case == "p7_48":
        M = A.generate(7, 48)
    elif case == "a27_20":
        M = A.generate(27, 20)
    else:
        keep = W.circuit_csr(60000)
        M = keep.mat
    return M, keep


def _same(M1, M2):
    a, b = A.csr_arrays(M1), A.csr_arrays(M2)
    return (M1.num_rows, M1.num_cols, M1.num_nnzs) == (M2.num_rows, M2.num_cols, M2.num_nnzs) and all(
        np.array_equal(x.view(np.uint8), y.view(np.uint8)) for x, y in zip(a, b))


@pytest.mark.parametrize("case", ["p7_32", "p7_48", "a27_20", "circ60k", "bus"])
@pytest.mark.parametrize("cfgs", ["4", "2", "1", "0"])
def test_rap_levels_bitwise(case, cfgs, monkeypatch):
    monkeypatch.setenv("SSS_HIP_RAP_CFGS", cfgs)   # fewer device tables: more rows retried / on the host
    M, keep = _mats(case)
    H = build_hierarchy(M, quiet_ctx)
    lib = A.lib()
    for l in range(H.num_levels - 1):
        L = H.level(l)
        Ch = lib.SSS_blas_mat_rap(C.byref(L.R), C.byref(L.A), C.byref(L.P))
        Cg = A.SSS_MAT()
        assert lib.sss_hip_rap(C.byref(L.R), C.byref(L.A), C.byref(L.P), C.byref(Cg)) == 0
        try:
            assert _same(Cg, Ch), (case, cfgs, l)
            assert _same(Cg, H.level(l + 1).A) or l + 2 == H.num_levels, (case, l)
        finally:
            lib.SSS_mat_destroy(C.byref(Cg))
            lib.SSS_mat_destroy(C.byref(Ch))
    del keep


def _digest(H) -> str:
    h = hashlib.sha256()
    for l in range(H.num_levels):
        for arr in A.csr_arrays(H.level(l).A):
            h.update(arr.tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("case", ["p7_48", "a27_20", "circ60k"])
def test_setup_with_gpu_rap_same_hierarchy(case, monkeypatch):
    """SSS_amg_setup with every level's product on the GPU (SSS_SETUP_GPU_RAP_MIN=0) builds the
    hierarchy the host products build, bit for bit."""
    M, keep = _mats(case)
    monkeypatch.setenv("SSS_SETUP_GPU_RAP", "0")
    d_host = _digest(build_hierarchy(M, quiet_ctx))
    monkeypatch.setenv("SSS_SETUP_GPU_RAP", "1")
    monkeypatch.setenv("SSS_SETUP_GPU_RAP_MIN", "0")
    monkeypatch.setenv("SSS_SETUP_GPU_RAP_MAXROW", "100000")
    d_gpu = _digest(build_hierarchy(M, quiet_ctx))
    assert d_gpu == d_host
    del keep
