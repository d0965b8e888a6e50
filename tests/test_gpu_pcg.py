"""GPU tests of the AMG-preconditioned CG (sss_hip_pcg; SURVEY.md §8f row 4, an engine extension).

Checks: convergence to tol with fewer iterations than the stand-alone V-cycle iteration, the true
residual ||b - A x|| / ||b|| (host, oracle SpMV) below tol, run-to-run determinism (bitwise x),
and agreement with a numpy restatement of the same flexible PCG whose preconditioner is the
oracle's V-cycle in the same mode (iteration counts equal, residual histories within 1e-6).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import amg_amd as A
import oracle
from amg_amd._native import SSS_VEC, dptr
from conftest import build_hierarchy, device_mode_oracle_opts

pytestmark = pytest.mark.gpu

MODES = {   # engine mode -> oracle options of the same algorithm (None: read from the device's levels)
    "hybrid": (dict(smoother="hybrid", coarse="direct"), None),
    "exact": (dict(smoother="exact", coarse="krylov"), {}),
}


@pytest.fixture(scope="module")
def p32_h(quiet):
    return build_hierarchy(A.generate(7, 32), quiet)


@pytest.fixture(scope="module")
def a27_h(quiet):
    return build_hierarchy(A.generate(27, 16), quiet)


def _gpu_pcg(H, mode, tol, maxit=100):
    n = H.level(0).A.num_rows
    D = A.DeviceHierarchy(H, **MODES[mode][0])
    D.upload(0, "b", np.ones(n))
    D.upload(0, "x", np.zeros(n))
    its, hist = D.pcg(tol, maxit)
    x = D.download(0, "x")
    D.close()
    return its, hist, x


def _oracle_pcg(H, mode, tol, maxit=100):
    """numpy flexible CG (Polak-Ribiere), M^-1 = one oracle V-cycle on (r, 0)."""
    ora = oracle.load()
    kw = MODES[mode][1]
    o = oracle.opts(**(kw if kw is not None else device_mode_oracle_opts(H, **MODES[mode][0])))
    A0 = H.level(0).A
    n = A0.num_rows
    bvec, xv = np.zeros(n), np.zeros(n)
    H.mg.cg[0].b = SSS_VEC(n, dptr(bvec))
    H.mg.cg[0].x = SSS_VEC(n, dptr(xv))

    def M(r):
        bvec[:] = r
        xv[:] = 0.0
        ora.ora_cycle(C.byref(H.mg), C.byref(o))
        return xv.copy()

    def Ax(v):
        y = np.zeros(n)
        ora.ora_mv_mxy(C.byref(A0), dptr(v), dptr(y))
        return y

    b = np.ones(n)
    x = np.zeros(n)
    r = b - Ax(x)
    z = M(r)
    p = z.copy()
    rz = r @ z
    nb = np.linalg.norm(b)
    hist = []
    for _ in range(maxit):
        q = Ax(p)
        a = rz / (p @ q)
        x += a * p
        ro = r.copy()
        r -= a * q
        hist.append(np.linalg.norm(r) / nb)
        if hist[-1] < tol:
            break
        z = M(r)
        rzn = r @ z
        p = z + ((rzn - ro @ z) / rz) * p
        rz = rzn
    return len(hist), np.array(hist), x


@pytest.mark.parametrize("hname", ["p32_h", "a27_h"])
@pytest.mark.parametrize("mode", ["hybrid", "exact"])
def test_pcg_matches_restatement(request, hname, mode):
    H = request.getfixturevalue(hname)
    tol = H.pars.tol
    its, hist, x = _gpu_pcg(H, mode, tol)
    its_r, hist_r, x_r = _oracle_pcg(H, mode, tol)
    assert hist[-1] < tol
    assert its == its_r
    assert np.allclose(hist, hist_r, rtol=1e-6, atol=0)
    assert np.linalg.norm(x - x_r) <= 1e-6 * np.linalg.norm(x_r)


@pytest.mark.parametrize("mode", ["hybrid", "exact"])
def test_pcg_true_residual_and_speedup(p32_h, mode):
    H = p32_h
    A0 = H.level(0).A
    n = A0.num_rows
    its, hist, x = _gpu_pcg(H, mode, H.pars.tol)
    y = np.zeros(n)
    oracle.load().ora_mv_mxy(C.byref(A0), dptr(x), dptr(y))
    assert np.linalg.norm(np.ones(n) - y) / np.sqrt(n) < 10 * H.pars.tol
    # fewer iterations than the stand-alone V-cycle iteration of the same engine mode
    D = A.DeviceHierarchy(H, **MODES[mode][0])
    D.upload(0, "b", np.ones(n))
    D.upload(0, "x", np.zeros(n))
    cycles = 0
    while cycles < 100:
        D.cycle()
        cycles += 1
        if D.residual_norm() / np.sqrt(n) < H.pars.tol:
            break
    D.close()
    assert its < cycles


def test_pcg_deterministic(a27_h):
    _, h1, x1 = _gpu_pcg(a27_h, "hybrid", a27_h.pars.tol)
    _, h2, x2 = _gpu_pcg(a27_h, "hybrid", a27_h.pars.tol)
    assert np.array_equal(x1.view(np.uint64), x2.view(np.uint64))
    assert np.array_equal(h1, h2)
