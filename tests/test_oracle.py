"""CPU: the oracle (CPU restatement of the solve phase) + the host C setup, pinned against the
reference's known answers (tests/golden/golden.json "survey" section)."""
from __future__ import annotations

import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

import amg_amd as A
import oracle
from amg_amd._native import SSS_VEC, dptr
from conftest import build_hierarchy, oracle_solve, seq_sum

GOLD = json.loads((Path(__file__).resolve().parent / "golden" / "golden.json").read_text())["survey"]


@pytest.fixture(scope="module")
def bus_h(bus_matrix, quiet):
    return build_hierarchy(bus_matrix, quiet)


def test_bus_hierarchy(bus_h):
    g = GOLD["bus_levels"]
    assert [[bus_h.level(l).A.num_rows, bus_h.level(l).A.num_nnzs] for l in range(bus_h.num_levels)] == g["n_nnz"]
    for l in range(bus_h.num_levels - 1):
        L = bus_h.level(l)
        assert L.P.num_cols == g["nC"][l]
        assert L.P.num_nnzs == g["nnzP"][l]
        _, _, v = A.csr_arrays(L.A)
        assert "%.17g" % seq_sum(v) == g["sumA"][l]


def test_bus_history_byte_identical(bus_matrix, quiet):
    H = build_hierarchy(bus_matrix, quiet)
    n = bus_matrix.num_rows
    rtn, rel, ab = oracle_solve(H, np.ones(n), np.ones(n))
    g = GOLD["bus_history"]
    assert rtn.nits == len(g["relres"]) - 1
    assert ["%.6e" % r for r in rel] == g["relres"][1:]
    assert ["%.6e" % a for a in ab] == g["absres"][1:]


def test_bus_x_after_cycles_17_digits(bus_matrix, quiet):
    H = build_hierarchy(bus_matrix, quiet)
    n = bus_matrix.num_rows
    x, b = np.ones(n), np.ones(n)
    H.mg.cg[0].x = SSS_VEC(n, dptr(x))
    H.mg.cg[0].b = SSS_VEC(n, dptr(b))
    g = GOLD["bus_cycles"]
    o = oracle.opts()
    for c in range(3):
        oracle.load().ora_cycle(C.byref(H.mg), C.byref(o))
        assert "%.17g" % seq_sum(x) == g["sum_x"][c]
        assert "%.17g" % x[0] == g["x0"][c]


@pytest.mark.parametrize("n,key", [(16, "poisson16"), (32, "poisson32")])
def test_poisson_histories(n, key, quiet):
    H = build_hierarchy(A.generate(7, n), quiet)
    N = n ** 3
    rtn, rel, _ = oracle_solve(H, np.ones(N), np.ones(N))
    assert ["%.6e" % r for r in rel] == GOLD[key]["relres"]
    if "n_nnz" in GOLD[key]:
        assert [[H.level(l).A.num_rows, H.level(l).A.num_nnzs] for l in range(H.num_levels)] == GOLD[key]["n_nnz"]


def test_poisson64_cycle1_and_solve(quiet):
    g = GOLD["poisson64"]
    H = build_hierarchy(A.generate(7, 64), quiet)
    assert [H.level(l).P.num_cols for l in range(H.num_levels - 1)] == g["nC"]
    Lc = H.level(H.num_levels - 1).A
    assert [Lc.num_rows, Lc.num_nnzs] == g["coarsest"]
    N = 64 ** 3
    x, b = np.ones(N), np.ones(N)
    H.mg.cg[0].x = SSS_VEC(N, dptr(x))
    H.mg.cg[0].b = SSS_VEC(N, dptr(b))
    oracle.load().ora_cycle(C.byref(H.mg), C.byref(oracle.opts()))
    assert "%.17g" % seq_sum(x) == g["sum_x_cycle1"]
    H2 = build_hierarchy(A.generate(7, 64), quiet)
    rtn, rel, _ = oracle_solve(H2, np.ones(N), np.ones(N))
    assert rtn.nits == g["iterations"]
    assert "%.5e" % rel[-1] == g["final_relres"]


@pytest.mark.slow
def test_poisson128_solve(quiet):
    g = GOLD["poisson128"]
    H = build_hierarchy(A.generate(7, 128), quiet)
    Lc = H.level(H.num_levels - 1).A
    assert [Lc.num_rows, Lc.num_nnzs] == g["coarsest"]
    N = 128 ** 3
    rtn, rel, _ = oracle_solve(H, np.ones(N), np.ones(N))
    assert rtn.nits == g["iterations"]
    assert "%.5e" % rel[-1] == g["final_relres"]


def test_direct_coarse_reproduces_history(quiet):
    """an exact coarse solve reproduces the reference's Poisson history (same
    iteration count; the printed 7th digit may move, as the survey measured at 256^3)."""
    H = build_hierarchy(A.generate(7, 32), quiet)
    N = 32 ** 3
    _, rel, _ = oracle_solve(H, np.ones(N), np.ones(N), coarse_mode=1)
    ref = np.array([float(r) for r in GOLD["poisson32"]["relres"]])
    assert len(rel) == len(ref)
    assert np.allclose(rel, ref, rtol=2e-6, atol=0)


def test_row_cap_as_shipped_identical_below_cap(bus_matrix, quiet):
    """Below 4,096 rows the as-shipped <<<64,64>>> cap is inactive."""
    H = build_hierarchy(bus_matrix, quiet)
    n = bus_matrix.num_rows
    _, rel_capped, _ = oracle_solve(H, np.ones(n), np.ones(n), row_cap=4096)
    assert ["%.6e" % r for r in rel_capped] == GOLD["bus_history"]["relres"][1:]


def test_cf_jacobi_converges(quiet):
    H = build_hierarchy(A.generate(7, 32), quiet)
    N = 32 ** 3
    rtn, rel, _ = oracle_solve(H, np.ones(N), np.ones(N), smoother=1, coarse_mode=1)
    assert rel[-1] < 1e-6 and rtn.nits <= len(GOLD["poisson32"]["relres"]) + 2
