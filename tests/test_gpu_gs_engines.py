"""GPU: the one-launch exact GS-CF engines (amg_amd/csrc/sss_gs_persist.hip) against the oracle.

Every exact GS-CF pass with intra-class chains runs as one launch per pass -- on one CU ("cu") or as
chip-wide dataflow ("flow") -- instead of one launch per DAG depth ("launch").  All three must be
bitwise identical to the sequential reference smoother (Solve/SSS_smooth.c:4-87, oracle
ora_smoother_pre/post) on every level, and whole parity-mode solves must give the reference's x bit
for bit.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import amg_amd as A
import oracle
from amg_amd._native import SSS_SMTR
from conftest import build_hierarchy, oracle_solve, vec

pytestmark = pytest.mark.gpu

ENGINES = {"launch": 0, "flow": 1, "cu": 2}


@pytest.fixture(scope="module")
def bus_h(bus_matrix, quiet):
    return build_hierarchy(bus_matrix, quiet)


@pytest.fixture(scope="module")
def p32_h(quiet):
    return build_hierarchy(A.generate(7, 32), quiet)


@pytest.fixture(scope="module")
def a27_h(quiet):
    return build_hierarchy(A.generate(27, 16), quiet)


@pytest.fixture(scope="module")
def p64_h(quiet):
    return build_hierarchy(A.generate(7, 64), quiet)


@pytest.fixture(params=list(ENGINES))
def engine(request, monkeypatch):
    monkeypatch.setenv("SSS_HIP_GS_ENGINE", request.param)
    return request.param


def _smtr(M, b, x, mark, sweeps, post, smoother=2):
    s = SSS_SMTR()
    s.smoother = smoother
    s.A = C.pointer(M)
    s.b = C.pointer(vec(b))
    s.x = C.pointer(vec(x))
    s.nsweeps = sweeps
    s.istart, s.iend, s.istep = 0, M.num_rows - 1, -1 if post else 1
    s.cf_order = 1
    s.ordering = mark
    return s


def _check_engines(D, H, engine):
    used = set()
    for l in range(H.num_levels - 1):
        info = D.level_info(l)
        assert info.gs_stall == 0, f"level {l}: a one-launch pass gave up waiting"
        for e, depth in ((info.gs_engine_f, info.dag_f), (info.gs_engine_c, info.dag_c)):
            if depth > 1:
                used.add(e)
    if engine != "launch":
        assert used <= {0, ENGINES[engine]}
        assert ENGINES[engine] in used or not used


@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h"])
def test_level_smoothers_bitwise(request, hname, engine):
    H = request.getfixturevalue(hname)
    ora = oracle.load()
    D = A.DeviceHierarchy(H, smoother="exact", coarse="krylov")
    rng = np.random.default_rng(31)
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
                sr = _smtr(L.A, b, xr, L.cfmark.d, sweeps, post)
                (ora.ora_smoother_post if post else ora.ora_smoother_pre)(C.byref(sr))
                assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64)), (hname, l, post, engine)
        _check_engines(D, H, engine)
    finally:
        D.close()


@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h", "p64_h"])
def test_parity_solve_bitwise(request, hname, engine):
    H = request.getfixturevalue(hname)
    n = H.level(0).A.num_rows
    rtn, rel_r, _ = oracle_solve(H, np.ones(n), x_r := np.ones(n))
    D = A.DeviceHierarchy(H, smoother="exact", coarse="krylov")
    try:
        D.upload(0, "b", np.ones(n))
        D.upload(0, "x", np.ones(n))
        rel = []
        for _ in range(len(rel_r)):
            D.cycle()
            rel.append(D.residual_norm() / np.sqrt(n))
        x_g = D.download(0, "x")
        _check_engines(D, H, engine)
    finally:
        D.close()
    assert np.array_equal(x_g.view(np.uint64), x_r.view(np.uint64))
    assert np.allclose(rel, rel_r, rtol=1e-13, atol=0)


def test_repeated_launches_stay_bitwise(p32_h, monkeypatch):
    """Epoch bookkeeping across many launches (graph replays included): 12 V-cycles per engine
    give the same iterate as the per-depth launches."""
    n = p32_h.level(0).A.num_rows
    out = {}
    for eng in ENGINES:
        monkeypatch.setenv("SSS_HIP_GS_ENGINE", eng)
        D = A.DeviceHierarchy(p32_h, smoother="exact", coarse="direct")
        try:
            D.upload(0, "b", np.ones(n))
            D.upload(0, "x", np.ones(n))
            for _ in range(12):
                D.cycle()
            out[eng] = D.download(0, "x")
            _check_engines(D, p32_h, eng)
        finally:
            D.close()
    for eng in ("flow", "cu"):
        assert np.array_equal(out[eng].view(np.uint64), out["launch"].view(np.uint64)), eng


# ---------------------------------------------------------------- natural-order GS (row a5)
def _natural(H):
    """The hierarchy with the reference's cf_order = 0 (SSS_amg_smoother_pre/post then call
    SSS_amg_smoother_gs, Solve/SSS_smooth.c:171-176, 256-260)."""
    H.mg.pars.cf_order = 0
    return H


@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h"])
def test_natural_gs_levels_bitwise(request, hname, engine):
    H = _natural(request.getfixturevalue(hname))
    ora = oracle.load()
    D = A.DeviceHierarchy(H, smoother="exact", coarse="krylov")
    rng = np.random.default_rng(41)
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
                sr = _smtr(L.A, b, xr, L.cfmark.d, sweeps, post)
                sr.cf_order = 0
                (ora.ora_smoother_post if post else ora.ora_smoother_pre)(C.byref(sr))
                assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64)), (hname, l, post, engine)
            info = D.level_info(l)
            assert info.gs_stall == 0
    finally:
        D.close()
        H.mg.pars.cf_order = 1


@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h"])
def test_natural_gs_solve_bitwise(request, hname, engine):
    H = _natural(request.getfixturevalue(hname))
    try:
        n = H.level(0).A.num_rows
        rtn, rel_r, _ = oracle_solve(H, np.ones(n), x_r := np.ones(n))
        D = A.DeviceHierarchy(H, smoother="exact", coarse="krylov")
        try:
            D.upload(0, "b", np.ones(n))
            D.upload(0, "x", np.ones(n))
            rel = []
            for _ in range(len(rel_r)):
                D.cycle()
                rel.append(D.residual_norm() / np.sqrt(n))
            x_g = D.download(0, "x")
        finally:
            D.close()
        assert np.array_equal(x_g.view(np.uint64), x_r.view(np.uint64))
        assert np.allclose(rel, rel_r, rtol=1e-13, atol=0)
    finally:
        H.mg.pars.cf_order = 1


@pytest.mark.parametrize("istart,iend,istep", [(0, -1, 1), (0, -1, -1), (5, 40, 1), (7, 30, -1), (30, 7, 1)])
def test_natural_gs_host_entry(p32_h, istart, iend, istep):
    """SSS_amg_smoother_pre/post's device entry with cf_order = 0 (any contiguous row range,
    either direction; crossed bounds run no row, as the reference's loops)."""
    ora = oracle.load()
    L = p32_h.level(1)
    n = L.A.num_rows
    iend = n - 1 if iend < 0 else iend
    rng = np.random.default_rng(istart + 3 * iend)
    for post in (False, True):
        b = rng.standard_normal(n)
        x0 = rng.standard_normal(n)
        xg, xr = x0.copy(), x0.copy()
        sg = _smtr(L.A, b, xg, L.cfmark.d, 2, post)
        sr = _smtr(L.A, b, xr, L.cfmark.d, 2, post)
        for s_ in (sg, sr):
            s_.cf_order = 0
            s_.istart, s_.iend, s_.istep = istart, iend, istep
        assert A.lib().sss_hip_host_smooth(C.byref(sg), int(post)) == 0
        (ora.ora_smoother_post if post else ora.ora_smoother_pre)(C.byref(sr))
        assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64)), (istart, iend, istep, post)


@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h"])
@pytest.mark.parametrize("smoother,coarse", [("exact", "krylov"), ("exact", "direct")])
def test_w_cycle_bitwise(request, hname, smoother, coarse):
    """cycle_type = 2 (the W-cycle branch of SSS_amg_cycle, Solve/SSS_cycle.cu:959-966: a level
    re-descends until it has been visited cycle_type times) -- x bitwise the oracle's."""
    H = request.getfixturevalue(hname)
    H.mg.pars.cycle_type = 2
    try:
        n = H.level(0).A.num_rows
        kw = {} if coarse == "krylov" else {"coarse_mode": 1}
        rtn, rel_r, _ = oracle_solve(H, np.ones(n), x_r := np.ones(n), **kw)
        D = A.DeviceHierarchy(H, smoother=smoother, coarse=coarse)
        try:
            D.upload(0, "b", np.ones(n))
            D.upload(0, "x", np.ones(n))
            rel = []
            for _ in range(len(rel_r)):
                D.cycle()
                rel.append(D.residual_norm() / np.sqrt(n))
            x_g = D.download(0, "x")
        finally:
            D.close()
        if coarse == "krylov":
            assert np.array_equal(x_g.view(np.uint64), x_r.view(np.uint64))
            assert np.allclose(rel, rel_r, rtol=1e-13, atol=0)
        else:   # explicit inverse vs the oracle's dense LU: same iterates to rounding (1138_bus is
            # ill-conditioned: the late residuals carry that rounding at ~1e-7 relative)
            assert np.linalg.norm(x_g - x_r) <= 1e-9 * np.linalg.norm(x_r)
            assert np.allclose(rel, rel_r, rtol=1e-4, atol=0)
    finally:
        H.mg.pars.cycle_type = 1


# ---------------------------------------------------------------- dictionary tiles
@pytest.mark.parametrize("hname", ["p32_h", "a27_h", "p64_h"])
@pytest.mark.parametrize("smoother,coarse", [("exact", "krylov"), ("hybrid", "direct")])
def test_dictionary_tiles_bitwise(request, hname, smoother, coarse, monkeypatch):
    """A_l stored as dictionary ELL rows (1 B per entry: offset and value indices into per-block
    dictionaries, one thread per row), as dictionary tiles (4 B per entry) or as value-dictionary
    sorted tiles (5 B: the sorted tile slot plus a value index) gives the iterates of the plain
    column-sorted tiles bit for bit, and the stencil levels do take that storage: level 0 of 7-pt
    the ELL rows (dictionary tiles with ELL off), the relabeled Galerkin levels of 7-pt 64^3
    (offsets too many for a dictionary, at most 8 values per block) the value dictionaries."""
    H = request.getfixturevalue(hname)
    n = H.level(0).A.num_rows
    out, fmt = {}, {}
    for mode, env in (("ell", {"SSS_HIP_DICT": "1", "SSS_HIP_ELL": "1"}),
                      ("tiles", {"SSS_HIP_DICT": "1", "SSS_HIP_ELL": "0"}),
                      ("none", {"SSS_HIP_DICT": "0", "SSS_HIP_ELL": "0"})):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        D = A.DeviceHierarchy(H, smoother=smoother, coarse=coarse)
        try:
            D.upload(0, "b", np.ones(n))
            D.upload(0, "x", np.ones(n))
            rel = []
            for _ in range(6):
                D.cycle()
                rel.append(D.residual_norm())
            out[mode] = (D.download(0, "x"), rel)
            fmt[mode] = [D.level_info(l).a_format for l in range(H.num_levels - 1)]
        finally:
            D.close()
    if hname != "a27_h":
        assert fmt["ell"][0] & 64, fmt
        assert fmt["tiles"][0] & 2 and not fmt["tiles"][0] & 64, fmt
    assert fmt["tiles"][0] & 2 or hname == "a27_h", fmt
    if hname == "p64_h":
        assert any(f & 3 == 3 for f in fmt["tiles"][1:]), fmt
    assert not any(f & 66 for f in fmt["none"])
    for mode in ("ell", "tiles"):
        assert np.array_equal(out[mode][0].view(np.uint64), out["none"][0].view(np.uint64)), mode
        assert out[mode][1] == out["none"][1], mode
