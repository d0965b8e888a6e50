"""GPU tests of the free summation order (sss_hip_opts.sum_order = 1, throughput mode).

On long-row levels (>= SSS_HIP_FREE_MIN entries per row on average) the free order sums each
row with a whole wave in a fixed tree order over a column-sorted copy of the row
(sss_spmv_dev.hpp wave_row_sum), or -- levels with enough rows -- G = 4 or 8 neighbouring rows
merged into one column-sorted list summed by one wave (merged_sums), instead of the reference's
sequential CSR order.  The result is
deterministic but not bitwise the oracle's, so the checks here are the SURVEY.md §8c ladder's
reordered-summation rows:
  * one smoother call per level (C/F-Jacobi and two-stage GS-CF, every level forced onto the
    wave kernels): ||x_gpu - x_oracle|| / ||x_oracle|| <= 1e-12;
  * whole solve (hybrid smoother, direct coarse solve): the same iteration count as the
    stored-order run, per-iteration relres within 1e-8 relative, final relres < tol;
  * run-to-run determinism: two free-order solves are bitwise identical.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import amg_amd as A
import oracle
from amg_amd._native import dptr
from conftest import build_hierarchy

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def p32_h(quiet):
    return build_hierarchy(A.generate(7, 32), quiet)


@pytest.fixture(scope="module")
def a27_h(quiet):
    return build_hierarchy(A.generate(27, 16), quiet)


@pytest.fixture(params=["wave", "merged4", "merged8", "merged4w1", "merged8w2"])
def all_wave(request, monkeypatch):
    """every matrix of the hierarchy on the free-order kernels: wave per row (tree sum over the
    column-sorted row), or merged row groups of 4 / 8 rows (sss_spmv_dev.hpp merged_sums) with
    4 (default for these sizes), 1 or 2 waves per group"""
    monkeypatch.setenv("SSS_HIP_WAVE_MIN", "1")
    monkeypatch.setenv("SSS_HIP_FREE_MIN", "1")
    if request.param == "wave":
        monkeypatch.setenv("SSS_HIP_MERGE_MIN_ROWS", str(1 << 30))
    else:
        monkeypatch.setenv("SSS_HIP_MERGE_MIN_ROWS", "1")
        monkeypatch.setenv("SSS_HIP_MERGE_G", request.param[6])
        monkeypatch.setenv("SSS_HIP_MERGE_W", request.param[8] if "w" in request.param else "4")
    return request.param


@pytest.mark.parametrize("hname", ["p32_h", "a27_h"])
@pytest.mark.parametrize("inner", [0, 1])
def test_free_order_smoothers_close(request, hname, inner, all_wave):
    H = request.getfixturevalue(hname)
    ora = oracle.load()
    D = A.DeviceHierarchy(H, smoother="jacobi", coarse="direct", relabel=1, inner=inner, inner_from=0,
                          sum_order=1)
    rng = np.random.default_rng(5)
    try:
        for l in range(H.num_levels - 1):
            L = H.level(l)
            n = L.A.num_rows
            for post in (False, True):
                b = rng.standard_normal(n)
                x0 = rng.standard_normal(n)
                D.upload(l, "b", b)
                D.upload(l, "x", x0)
                D.smooth(l, post)
                xg = D.download(l, "x")
                xr = x0.copy()
                sweeps = H.pars.post_iter if post else H.pars.pre_iter
                if inner > 0:
                    ora.ora_cf_twostage(dptr(xr), C.byref(L.A), dptr(b), sweeps, L.cfmark.d, inner)
                else:
                    ora.ora_cf_jacobi(dptr(xr), C.byref(L.A), dptr(b), sweeps, L.cfmark.d)
                err = np.linalg.norm(xg - xr) / np.linalg.norm(xr)
                assert err <= 1e-12, (l, post, err)
    finally:
        D.close()


def _history(H, sum_order, max_it=60):
    n = H.level(0).A.num_rows
    D = A.DeviceHierarchy(H, smoother="hybrid", coarse="direct", sum_order=sum_order)
    D.upload(0, "b", np.ones(n))
    D.upload(0, "x", np.ones(n))
    rel = []
    for _ in range(max_it):
        D.cycle()
        rel.append(D.residual_norm() / np.sqrt(n))
        if rel[-1] < H.pars.tol:
            break
    x = D.download(0, "x")
    D.close()
    return np.array(rel), x


@pytest.mark.parametrize("hname", ["p32_h", "a27_h"])
def test_free_order_solve_matches_stored_order(request, hname, all_wave):
    H = request.getfixturevalue(hname)
    rel_s, x_s = _history(H, 0)
    rel_f, x_f = _history(H, 1)
    assert len(rel_f) == len(rel_s)
    assert rel_f[-1] < H.pars.tol
    assert np.allclose(rel_f, rel_s, rtol=1e-8, atol=0)
    assert np.linalg.norm(x_f - x_s) <= 1e-10 * np.linalg.norm(x_s)


def test_free_order_is_deterministic(a27_h, all_wave):
    rel1, x1 = _history(a27_h, 1, max_it=5)
    rel2, x2 = _history(a27_h, 1, max_it=5)
    assert np.array_equal(x1.view(np.uint64), x2.view(np.uint64))
    assert np.array_equal(rel1, rel2)


@pytest.mark.parametrize("hname", ["p32_h", "a27_h"])
def test_sorted_tiles_bitwise_neutral(request, hname):
    """Column-sorted tile staging changes only the order the products are FORMED in, never the
    order they are added: iterates with it on and off are bitwise identical (exact and hybrid)."""
    H = request.getfixturevalue(hname)
    n = H.level(0).A.num_rows
    for smoother, coarse in (("exact", "krylov"), ("hybrid", "direct")):
        xs = []
        for st in (0, 1):
            D = A.DeviceHierarchy(H, smoother=smoother, coarse=coarse, sorted_tiles=st, formats="full")
            D.upload(0, "b", np.ones(n))
            D.upload(0, "x", np.ones(n))
            for _ in range(3):
                D.cycle()
            xs.append(D.download(0, "x"))
            D.close()
        assert np.array_equal(xs[0].view(np.uint64), xs[1].view(np.uint64)), smoother
