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

# "fused": the flow engine with every pass of a smoother call in one launch (level_info reports 3)
ENGINES = {"launch": 0, "flow": 1, "cu": 2, "fused": 3}


def _set_engine(mp, name):
    mp.setenv("SSS_HIP_GS_ENGINE", "flow" if name == "fused" else name)
    mp.setenv("SSS_HIP_GS_FUSED", "1" if name == "fused" else "0")


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
    _set_engine(monkeypatch, request.param)
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
    if engine == "fused":   # a level whose passes are not both flow passes keeps them
        assert used <= {0, 1, 3}
    elif engine != "launch":
        assert used <= {0, ENGINES[engine]}
        assert ENGINES[engine] in used or not used
    return used


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
        _set_engine(monkeypatch, eng)
        D = A.DeviceHierarchy(p32_h, smoother="exact", coarse="direct")
        try:
            D.upload(0, "b", np.ones(n))
            D.upload(0, "x", np.ones(n))
            for _ in range(12):
                D.cycle()
            out[eng] = D.download(0, "x")
            used = _check_engines(D, p32_h, eng)
            if eng == "fused":
                assert 3 in used, used
        finally:
            D.close()
    for eng in ("flow", "cu", "fused"):
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


def _nonsym_upwind(nx: int, seed: int):
    """Structurally nonsymmetric 2-D operator: 5-point upwind convection-diffusion on an nx*nx
    grid, with the east coupling dropped on a random third of the rows (so the same-pass coupling
    of the one-launch engines is not symmetric and they must not take the pass)."""
    rng = np.random.default_rng(seed)
    rp, ci, v = [0], [], []
    for j in range(nx):
        for i in range(nx):
            r = i + nx * j
            ent = []
            if j > 0:
                ent.append((r - nx, -1.5))
            if i > 0:
                ent.append((r - 1, -1.25))
            ent.append((r, 4.5 + 0.1 * rng.random()))
            if i + 1 < nx and rng.random() > 1 / 3:
                ent.append((r + 1, -0.5))
            if j + 1 < nx:
                ent.append((r + nx, -0.75))
            for c, a in ent:
                ci.append(c)
                v.append(a)
            rp.append(len(ci))
    return A.NumpyCSR(np.array(rp), np.array(ci), np.array(v))


@pytest.mark.parametrize("istart,iend,istep", [(0, -1, 1), (0, -1, -1), (17, 900, 1)])
def test_natural_gs_nonsymmetric_bitwise(istart, iend, istep, engine):
    """Natural-order GS (x_i = t * d with the carried reciprocal, Solve/SSS_smooth.c:90-137) on a
    structurally nonsymmetric matrix: whichever engine is asked for, the pass falls back to a form
    that multiplies by the reciprocal -- bitwise the oracle in both directions."""
    ora = oracle.load()
    M = _nonsym_upwind(40, 5)
    n = M.mat.num_rows
    iend = n - 1 if iend < 0 else iend
    mark = np.zeros(n, np.int32)
    rng = np.random.default_rng(istart + iend)
    for post in (False, True):
        b = rng.standard_normal(n)
        x0 = rng.standard_normal(n)
        xg, xr = x0.copy(), x0.copy()
        sg = _smtr(M.mat, b, xg, mark.ctypes.data_as(C.POINTER(C.c_int)), 2, post)
        sr = _smtr(M.mat, b, xr, mark.ctypes.data_as(C.POINTER(C.c_int)), 2, post)
        for s_ in (sg, sr):
            s_.cf_order = 0
            s_.istart, s_.iend, s_.istep = istart, iend, istep
        assert A.lib().sss_hip_host_smooth(C.byref(sg), int(post)) == 0
        (ora.ora_smoother_post if post else ora.ora_smoother_pre)(C.byref(sr))
        assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64)), (istart, iend, istep, post, engine)


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
    dictionaries, one thread per row), as column ELL rows (4 B per entry: explicit column and a
    value index, one thread per row), as dictionary tiles (4 B per entry) or as value-dictionary
    sorted tiles (5 B: the sorted tile slot plus a value index) gives the iterates of the plain
    column-sorted tiles bit for bit, and the stencil levels do take that storage: level 0 of 7-pt
    the dictionary ELL rows (dictionary tiles with both ELLs off, column ELL with only the
    dictionary ELL off -- every relaxation mode of the exact level-0 passes), the relabeled Galerkin
    levels of 7-pt (offsets too many for a 1-byte dictionary, at most 8 values per block) the column
    ELL, or the value dictionaries with it off."""
    H = request.getfixturevalue(hname)
    n = H.level(0).A.num_rows
    out, fmt = {}, {}
    monkeypatch.setenv("SSS_HIP_FORMATS", "full")   # (the exact smoother's own default is plain tiles)
    for mode, env in (("ell", {"SSS_HIP_DICT": "1", "SSS_HIP_ELL": "1", "SSS_HIP_XELL": "1"}),
                      ("xell", {"SSS_HIP_DICT": "1", "SSS_HIP_ELL": "0", "SSS_HIP_XELL": "1"}),
                      ("tiles", {"SSS_HIP_DICT": "1", "SSS_HIP_ELL": "0", "SSS_HIP_XELL": "0"}),
                      ("none", {"SSS_HIP_DICT": "0", "SSS_HIP_ELL": "0", "SSS_HIP_XELL": "1"})):
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
        assert fmt["xell"][0] & 128, fmt
        assert fmt["ell"][1] & 128, fmt
        assert fmt["tiles"][0] & 2 and not fmt["tiles"][0] & 192, fmt
    assert fmt["tiles"][0] & 2 or hname == "a27_h", fmt
    if hname == "p64_h":
        assert any(f & 3 == 3 for f in fmt["tiles"][1:]), fmt
    assert not any(f & 194 for f in fmt["none"])
    for mode in ("ell", "xell", "tiles"):
        assert np.array_equal(out[mode][0].view(np.uint64), out["none"][0].view(np.uint64)), mode
        # the norm's partial sums follow the row blocking, which the column ELL sets to 256 rows:
        # the same squares, summed in another fixed order
        assert np.allclose(out[mode][1], out["none"][1], rtol=1e-14, atol=0), mode


# ---------------------------------------------------------------- a stalled pass fails loudly
def _flow_levels(D, H):
    return [l for l in range(H.num_levels - 1)
            if D.level_info(l).gs_engine_f or D.level_info(l).gs_engine_c]


def test_stall_fails_loudly(p32_h, monkeypatch):
    """A one-launch pass that gives up waiting (forced here: SSS_HIP_GS_SPIN < 0 makes every launch
    report a stall) invalidates the iterate: the residual norm that follows, the sync and the
    download all fail instead of returning a plausible residual over a wrong x -- and the error
    word is cleared on read, so the next check reports only new stalls."""
    monkeypatch.setenv("SSS_HIP_GS_SPIN", "-1")
    n = p32_h.level(0).A.num_rows
    D = A.DeviceHierarchy(p32_h, smoother="exact", coarse="krylov")
    try:
        assert _flow_levels(D, p32_h), "no one-launch pass on this hierarchy"
        D.upload(0, "b", np.ones(n))
        D.upload(0, "x", np.ones(n))
        D.cycle()
        with pytest.raises(RuntimeError, match="residual_norm"):
            D.residual_norm()
        D.sync()   # cleared by the read above, nothing new since
        D.cycle()
        with pytest.raises(RuntimeError, match="sync"):
            D.sync()
        D.cycle()
        with pytest.raises(RuntimeError, match="download"):
            D.download(0, "x")
    finally:
        D.close()


def test_tiny_spin_limit_never_silent(p32_h, monkeypatch):
    """With a spin limit of zero polls a pass gives up whenever a row's lower neighbour is not yet
    published: every outcome is either the reference's x bit for bit or a loud failure."""
    monkeypatch.setenv("SSS_HIP_GS_SPIN", "0")
    n = p32_h.level(0).A.num_rows
    _, rel_r, _ = oracle_solve(p32_h, np.ones(n), x_r := np.ones(n))
    D = A.DeviceHierarchy(p32_h, smoother="exact", coarse="krylov")
    stalled = False
    try:
        D.upload(0, "b", np.ones(n))
        D.upload(0, "x", np.ones(n))
        try:
            for _ in range(len(rel_r)):
                D.cycle()
                D.residual_norm()
            x_g = D.download(0, "x")
        except RuntimeError:
            stalled = True
    finally:
        D.close()
    if not stalled:
        assert np.array_equal(x_g.view(np.uint64), x_r.view(np.uint64))


def test_stall_exits_drop_in_cli(tmp_path):
    """The drop-in CLI (amg file.mtx) on a stalled pass: exit(ERROR_MISC) with a '### ERROR' line,
    no iteration row after the failure, as the reference's fatal paths (SSS_utils.c:16-94)."""
    import os
    import subprocess
    from conftest import BUS_MTX, ROOT
    exe = ROOT / "amg_amd" / "bin" / "amg"
    env = dict(os.environ, SSS_HIP_GS_SPIN="-1")
    r = subprocess.run([str(exe), str(BUS_MTX)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == (-14 & 0xFF), (r.returncode, r.stderr[-2000:])
    assert "### ERROR" in r.stdout and "stalled" in r.stderr
    rows = [l for l in r.stdout.splitlines() if l[:6].strip().isdigit() and "|" in l]
    assert len(rows) <= 1, rows   # only the iteration-0 row
    assert "AMG solve time" not in r.stdout


# ---------------------------------------------------------------- fused engine edge cases
def _sym_two_class(n: int, nf: int, seed: int):
    """Structurally symmetric random operator with F rows [0, nf) and C rows [nf, n) (the relabeled
    layout the one-launch engines need), couplings inside and across the classes, rows without a
    diagonal (stale divisor, Solve/SSS_smooth.c:30,46), a zero diagonal (|d| <= 1e-20: x_i kept)
    and a row with no off-diagonal entry at all."""
    rng = np.random.default_rng(seed)
    cols = [set() for _ in range(n)]
    for i in range(n):
        for j in rng.integers(0, n, 5).tolist():
            if j != i and i != 11 and j != 11:
                cols[i].add(j)
                cols[j].add(i)
    rp, ci, v = [0], [], []
    for i in range(n):
        ent = sorted(cols[i] | ({i} if i % 7 else set()))
        for c in ent:
            ci.append(c)
            v.append((0.0 if i == 40 else 6.0 + rng.random()) if c == i else -0.4 * rng.random() - 0.1)
        rp.append(len(ci))
    mark = np.array([0] * nf + [1] * (n - nf), np.int32)
    return A.NumpyCSR(np.array(rp), np.array(ci), np.array(v)), mark


@pytest.mark.parametrize("fused", ["0", "1"])
def test_fused_engine_edge_rows_bitwise(fused, monkeypatch):
    """Host smoother entry (no uploaded level: the fused depth is computed on the host) over a
    relabeled two-class operator with missing and zero diagonals and an isolated row: 1, 2 and 3
    sweeps (the fused plan serves the 2-sweep calls), both directions, bitwise the oracle."""
    monkeypatch.setenv("SSS_HIP_GS_ENGINE", "flow")
    monkeypatch.setenv("SSS_HIP_GS_FUSED", fused)
    ora = oracle.load()
    M, mark = _sym_two_class(600, 350, 9)
    n = M.mat.num_rows
    rng = np.random.default_rng(17)
    for sweeps in (1, 2, 3):
        for post in (False, True):
            b = rng.standard_normal(n)
            x0 = rng.standard_normal(n)
            xg, xr = x0.copy(), x0.copy()
            sg = _smtr(M.mat, b, xg, mark.ctypes.data_as(C.POINTER(C.c_int)), sweeps, post)
            sr = _smtr(M.mat, b, xr, mark.ctypes.data_as(C.POINTER(C.c_int)), sweeps, post)
            assert A.lib().sss_hip_host_smooth(C.byref(sg), int(post)) == 0
            (ora.ora_smoother_post if post else ora.ora_smoother_pre)(C.byref(sr))
            assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64)), (sweeps, post, fused)


@pytest.mark.parametrize("nonfinite", [False, True])
@pytest.mark.parametrize("smoother", [2, 1])   # SSS_SM_GS (exact GS-CF), SSS_SM_JACOBI (C/F-Jacobi)
@pytest.mark.parametrize("fused", ["0", "1"])
def test_host_smooth_zero_iterate(fused, smoother, nonfinite, monkeypatch):
    """A zero iterate (every bit of x zero) takes the zero-iterate forms: the fused engine's reduced
    sweep-0 rows and the C/F-Jacobi first pass without the matrix.  Their exactness rests on two
    guards, both forced here: b_i = -0.0 on many rows (the dropped products (+-0) would otherwise
    turn -0.0 into +0.0 in the reference's chain) and, in the second case, a non-finite entry
    (inf * 0 = NaN must reach the rows that read it: the plans then keep every product).  Bitwise
    the oracle's smoother for 1, 2 and 3 sweeps, both directions."""
    monkeypatch.setenv("SSS_HIP_GS_ENGINE", "flow")
    monkeypatch.setenv("SSS_HIP_GS_FUSED", fused)
    ora = oracle.load()
    M, mark = _sym_two_class(600, 350, 9)
    n = M.mat.num_rows
    if nonfinite:
        rp = M.rp
        M.v[rp[100] + (1 if M.ci[rp[100]] == 100 else 0)] = np.inf   # an off-diagonal entry of row 100
    rng = np.random.default_rng(23)
    mk = mark.ctypes.data_as(C.POINTER(C.c_int))
    for sweeps in (1, 2, 3):
        for post in (False, True):
            b = rng.standard_normal(n)
            b[::5] = -0.0
            b[1::11] = 0.0
            xg, xr = np.zeros(n), np.zeros(n)
            assert A.lib().sss_hip_host_smooth(C.byref(_smtr(M.mat, b, xg, mk, sweeps, post, smoother)), int(post)) == 0
            (ora.ora_smoother_post if post else ora.ora_smoother_pre)(C.byref(_smtr(M.mat, b, xr, mk, sweeps, post,
                                                                                     smoother)))
            # NaNs at the same rows (their sign bit is the hardware's: x86 and gfx950 differ), every
            # other value bitwise
            ng, nr = np.isnan(xg), np.isnan(xr)
            assert np.array_equal(ng, nr), (sweeps, post, fused, smoother)
            assert np.array_equal(xg[~ng].view(np.uint64), xr[~nr].view(np.uint64)), (sweeps, post, fused, smoother)
            assert (~np.isfinite(xr)).any() == nonfinite


@pytest.mark.parametrize("fused", ["0", "1"])
def test_host_smooth_stall_fails(fused, monkeypatch):
    """The host smoother entry (SSS_amg_smoother_pre/post) on a stalled one-launch pass or fused
    call (forced: SSS_HIP_GS_SPIN < 0) returns the stall error instead of a wrong x, and the stall
    word is cleared: the same call without the hook succeeds and is bitwise the oracle."""
    monkeypatch.setenv("SSS_HIP_GS_ENGINE", "flow")
    monkeypatch.setenv("SSS_HIP_GS_FUSED", fused)
    ora = oracle.load()
    M, mark = _sym_two_class(600, 350, 9)
    n = M.mat.num_rows
    rng = np.random.default_rng(5)
    b = rng.standard_normal(n)
    x0 = rng.standard_normal(n)
    mk = mark.ctypes.data_as(C.POINTER(C.c_int))
    monkeypatch.setenv("SSS_HIP_GS_SPIN", "-1")
    xg = x0.copy()
    assert A.lib().sss_hip_host_smooth(C.byref(_smtr(M.mat, b, xg, mk, 2, False)), 0) == -14   # ERROR_MISC
    monkeypatch.delenv("SSS_HIP_GS_SPIN")
    xg, xr = x0.copy(), x0.copy()
    assert A.lib().sss_hip_host_smooth(C.byref(_smtr(M.mat, b, xg, mk, 2, False)), 0) == 0
    ora.ora_smoother_pre(C.byref(_smtr(M.mat, b, xr, mk, 2, False)))
    assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64))


@pytest.mark.parametrize("depth_form", ["gpu", "host"])
def test_fused_depth_forms(p32_h, depth_form, monkeypatch):
    """The fused plan's ticket order (fused-DAG depth) computed on the GPU per depth group or on the
    host in one serial pass: either is a topological order -- no stall, the reference's x bit for bit."""
    monkeypatch.setenv("SSS_HIP_GS_ENGINE", "flow")
    monkeypatch.setenv("SSS_HIP_GS_FUSED", "1")
    monkeypatch.setenv("SSS_HIP_FUSED_DEPTH", depth_form)
    n = p32_h.level(0).A.num_rows
    rtn, rel_r, _ = oracle_solve(p32_h, np.ones(n), x_r := np.ones(n))
    D = A.DeviceHierarchy(p32_h, smoother="exact", coarse="krylov")
    try:
        D.upload(0, "b", np.ones(n))
        D.upload(0, "x", np.ones(n))
        for _ in range(len(rel_r)):
            D.cycle()
        x_g = D.download(0, "x")
        used = _check_engines(D, p32_h, "fused")
        assert 3 in used
    finally:
        D.close()
    assert np.array_equal(x_g.view(np.uint64), x_r.view(np.uint64))


@pytest.mark.parametrize("shards", ["1", "3", "8"])
@pytest.mark.parametrize("lanes", ["2", "4", "16", "64"])
@pytest.mark.parametrize("hname", ["p32_h", "a27_h"])
def test_fused_lanes_per_row(request, hname, lanes, shards, monkeypatch):
    """Every lanes-per-row width of the fused engine (the planner picks 2 only on the widest levels
    of short rows, which the test sizes never reach), with one, three or eight ticket counters: the
    reference's x bit for bit, no stall."""
    monkeypatch.setenv("SSS_HIP_GS_ENGINE", "flow")
    monkeypatch.setenv("SSS_HIP_GS_FUSED", "1")
    monkeypatch.setenv("SSS_HIP_FUSED_G", lanes)
    monkeypatch.setenv("SSS_HIP_FUSED_SHARDS", shards)
    H = request.getfixturevalue(hname)
    n = H.level(0).A.num_rows
    rtn, rel_r, _ = oracle_solve(H, np.ones(n), x_r := np.ones(n))
    D = A.DeviceHierarchy(H, smoother="exact", coarse="krylov")
    try:
        D.upload(0, "b", np.ones(n))
        D.upload(0, "x", np.ones(n))
        for _ in range(len(rel_r)):
            D.cycle()
        x_g = D.download(0, "x")
        assert 3 in _check_engines(D, H, "fused")
    finally:
        D.close()
    assert np.array_equal(x_g.view(np.uint64), x_r.view(np.uint64))


def test_fused_engine_used_and_matches_per_pass(p64_h, monkeypatch):
    """On 7-pt 64^3 every level whose two passes are flow passes runs fused (level_info 3/3), and a
    V-cycle sequence gives the per-pass engine's iterate and residual norms bit for bit."""
    n = p64_h.level(0).A.num_rows
    out = {}
    for fused in ("0", "1"):
        monkeypatch.setenv("SSS_HIP_GS_ENGINE", "flow")
        monkeypatch.setenv("SSS_HIP_GS_FUSED", fused)
        D = A.DeviceHierarchy(p64_h, smoother="exact", coarse="krylov")
        try:
            eng = [(D.level_info(l).gs_engine_f, D.level_info(l).gs_engine_c) for l in range(p64_h.num_levels - 1)]
            D.upload(0, "b", np.ones(n))
            D.upload(0, "x", np.ones(n))
            rel = []
            for _ in range(5):
                D.cycle()
                rel.append(D.residual_norm())
            out[fused] = (D.download(0, "x"), rel, eng)
            assert all(D.level_info(l).gs_stall == 0 for l in range(p64_h.num_levels - 1))
        finally:
            D.close()
    assert any(e == (3, 3) for e in out["1"][2]), out["1"][2]
    assert all(e != (3, 3) for e in out["0"][2])
    for e0, e1 in zip(out["0"][2], out["1"][2]):
        assert e1 == (3, 3) or e1 == e0
        if e0 == (1, 1):
            assert e1 == (3, 3)
    assert np.array_equal(out["0"][0].view(np.uint64), out["1"][0].view(np.uint64))
    assert out["0"][1] == out["1"][1]


@pytest.mark.parametrize("hname", ["p32_h", "a27_h"])
def test_exact_mirror_formats_lean_by_default(request, hname, monkeypatch):
    """The exact smoother's mirror stores every operator as plain CSR tiles (formats auto = lean:
    its cycle waits on the GS-CF chains, the formats only cost build time); full formats give the
    same iterates bit for bit."""
    monkeypatch.delenv("SSS_HIP_FORMATS", raising=False)
    H = request.getfixturevalue(hname)
    n = H.level(0).A.num_rows
    out, fmt = {}, {}
    for formats in (None, "full"):
        D = A.DeviceHierarchy(H, smoother="exact", coarse="krylov", formats=formats)
        try:
            fmt[formats] = [(D.level_info(l).a_format, D.level_info(l).r_format, D.level_info(l).p_format)
                            for l in range(H.num_levels - 1)]
            D.upload(0, "b", np.ones(n))
            D.upload(0, "x", np.ones(n))
            for _ in range(4):
                D.cycle()
            out[formats] = D.download(0, "x")
        finally:
            D.close()
    assert all((a | r | p) & 0xC3 == 0 for a, r, p in fmt[None]), fmt[None]   # no ELL / dictionary / sorted tiles
    assert any((a | r | p) & 0xC3 for a, r, p in fmt["full"]), fmt["full"]
    assert np.array_equal(out[None].view(np.uint64), out["full"].view(np.uint64))
