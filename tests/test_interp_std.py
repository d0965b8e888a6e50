"""Standard interpolation (pars.interp_type = intERP_STD, 2): the reference's non-default
interpolation, Setup/SSS_coarsen.c:633-725 (form_P_pattern_std) + Setup/SSS_inter.cu:550-715
(interp_STD).

* The pattern is pinned by the reference's own compiled SSS_coarsen.c (live where oracle/_ref was
  built, and by the committed `bus_coarsen_std` fixture everywhere).
* The weights: SSS_inter.cu is a CUDA unit and unbuildable here, so they are checked bit for bit
  against the oracle's sequential restatement (`ora_interp_std`, the reference's row loop with its
  shared scratch arrays) on the same pattern; the truncation after them is the same restatement.
* The solve phase needs nothing of its own: the GPU V-cycle over a standard-interpolation hierarchy
  is compared with the oracle's (`-m gpu`).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import amg_amd as A
import oracle
from amg_amd._native import SSS_IMAT, SSS_MAT, NumpyCSR, csr_arrays
from amg_amd.workloads import circuit_csr
from conftest import BUS_MTX, oracle_solve

HERE = Path(__file__).resolve().parent
REFG = json.loads((HERE / "golden" / "golden.json").read_text())["ref_units"]
needs_ref = pytest.mark.skipif(not oracle.REF_PATH.exists(), reason="reference units not built (no /root/reference)")
STD = 2


def ihash(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.int32).tobytes()).hexdigest()[:24]


def std_pars():
    p = A.default_pars()
    p.interp_type = STD
    return p


_keep = []   # NumpyCSR matrices whose buffers must outlive their SSS_MAT views


def matrix(gen):
    if gen == "bus":
        return A.read_mtx(BUS_MTX)
    if gen == "p7_12":
        return A.generate(7, 12)
    if gen == "a27_8":
        return A.generate(27, 8)
    if gen == "circuit":
        M = circuit_csr(3000)
        _keep.append(M)
        return M.mat
    raise ValueError(gen)


def coarsen(lib, M, pars, quiet):
    verts = lib.SSS_ivec_create(M.num_rows)
    P, S = SSS_MAT(), SSS_IMAT()
    with quiet():
        rc = lib.SSS_amg_coarsen(C.byref(M), C.byref(verts), C.byref(P), C.byref(S),
                                 C.cast(C.byref(pars), C.c_void_p) if lib is not A.lib() else C.byref(pars))
    mark = np.ctypeslib.as_array(verts.d, shape=(M.num_rows,)).copy()
    return rc, verts, mark, P, S


def test_std_pattern_golden(quiet):
    M = A.read_mtx(BUS_MTX)
    rc, _, mark, P, _ = coarsen(A.lib(), M, std_pars(), quiet)
    prp, pci, _ = csr_arrays(P)
    got = {"rc": rc, "mark": ihash(mark), "nC_col": P.num_cols, "n_c_points": int((mark == 1).sum()),
           "P_rp": ihash(prp), "P_ci": ihash(pci), "P_nnz": P.num_nnzs}
    assert got == REFG["bus_coarsen_std"]


@needs_ref
@pytest.mark.parametrize("gen", ["bus", "p7_12", "a27_8", "circuit"])
def test_std_pattern_vs_reference(gen, quiet):
    M = matrix(gen)
    r1, _, m1, P1, S1 = coarsen(A.lib(), M, std_pars(), quiet)
    r2, _, m2, P2, S2 = coarsen(oracle.load_ref(), M, std_pars(), quiet)
    assert r1 == r2 == 0
    assert np.array_equal(m1, m2)
    assert P1.num_cols == P2.num_cols
    for x, y in zip(csr_arrays(P1)[:2], csr_arrays(P2)[:2]):
        assert np.array_equal(x, y)
    # the strong-coupling matrix the interpolation reads
    assert S1.num_nnzs == S2.num_nnzs
    s1 = (np.ctypeslib.as_array(S1.row_ptr, shape=(S1.num_rows + 1,)), np.ctypeslib.as_array(S1.col_idx, shape=(S1.num_nnzs,)))
    s2 = (np.ctypeslib.as_array(S2.row_ptr, shape=(S2.num_rows + 1,)), np.ctypeslib.as_array(S2.col_idx, shape=(S2.num_nnzs,)))
    assert np.array_equal(s1[0], s2[0]) and np.array_equal(s1[1], s2[1])


@pytest.mark.parametrize("gen", ["bus", "p7_12", "a27_8", "circuit"])
def test_std_weights_vs_oracle(gen, quiet):
    M = matrix(gen)
    pars = std_pars()
    rc, verts, mark, P, S = coarsen(A.lib(), M, pars, quiet)
    assert rc == 0
    prp, pci, pv = csr_arrays(P)
    ref = NumpyCSR(prp, pci, pv, ncols=P.num_cols)   # the pattern, before the product fills it
    with quiet():
        A.lib().SSS_amg_interp(C.byref(M), C.byref(verts), C.byref(P), C.byref(S), C.byref(pars))
        oracle.load().ora_interp_std(C.byref(M), verts.d, C.byref(ref.mat), C.byref(S), pars.trunc_threshold)
    got = csr_arrays(P)
    want = (ref.rp[: ref.mat.num_rows + 1], ref.ci[: ref.mat.num_nnzs], ref.v[: ref.mat.num_nnzs])
    assert P.num_cols == ref.mat.num_cols and P.num_nnzs == ref.mat.num_nnzs
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    assert np.array_equal(got[2].view(np.uint64), want[2].view(np.uint64))


@pytest.mark.parametrize("gen", ["bus", "p7_12"])
def test_std_hierarchy_solves(gen, quiet):
    """The whole setup with interp_type 2, then the oracle's solve (reference semantics) to tol."""
    M = matrix(gen)
    with quiet():
        H = A.Hierarchy(M, std_pars())
    assert H.num_levels >= 2
    n = M.num_rows
    for l in range(H.num_levels - 1):
        L = H.level(l)
        assert L.P.num_rows == L.A.num_rows and L.P.num_cols == H.level(l + 1).A.num_rows
    rtn, rel, _ = oracle_solve(H, np.ones(n), np.ones(n))
    assert rel[-1] < H.pars.tol


# ---------------------------------------------------------------- GPU: the solve phase over it
@pytest.fixture(scope="module")
def std_hiers():
    hs = {}
    yield hs
    for H in hs.values():
        H.close()


@pytest.mark.gpu
@pytest.mark.parametrize("gen", ["bus", "p7_24", "a27_12"])
def test_gpu_std_solve_parity_mode(gen, quiet, std_hiers):
    M = A.read_mtx(BUS_MTX) if gen == "bus" else A.generate(7, 24) if gen == "p7_24" else A.generate(27, 12)
    with quiet():
        H = std_hiers.setdefault(gen, A.Hierarchy(M, std_pars()))
    n = M.num_rows
    rtn, rel_r, _ = oracle_solve(H, np.ones(n), x_r := np.ones(n))
    D = A.DeviceHierarchy(H, smoother="exact", coarse="krylov")
    try:
        D.upload(0, "b", np.ones(n))
        D.upload(0, "x", np.ones(n))
        rel_g = []
        for _ in range(len(rel_r)):
            D.cycle()
            rel_g.append(D.residual_norm() / np.sqrt(n))
        x_g = D.download(0, "x")
    finally:
        D.close()
    # the iterate is bitwise the oracle's; only the level-0 norm is reduced in tree order on the GPU
    assert np.array_equal(x_g.view(np.uint64), x_r.view(np.uint64))
    assert np.allclose(rel_g, rel_r, rtol=1e-13, atol=0)
