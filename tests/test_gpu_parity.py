"""GPU parity tests (run on the MI355X box: `pytest -m gpu`).

Every comparison is HIP path (through the C ABI of libsss_amg.so) vs the CPU oracle on the same
inputs.  Tolerance ladder:
  * SpMV / residual / restriction / prolongation and the exact GS-CF smoother: BITWISE;
  * coarse Krylov solve (sequential-order reductions on device): BITWISE;
  * whole solve, parity mode: identical iteration count, BITWISE x, per-iteration relres
    rel <= 1e-13 (the level-0 ||r|| is a fixed-order tree reduction);
  * whole solve, direct coarse: identical iteration count on Poisson, relres rel <= 1e-6 per row,
    final x rel <= 1e-6.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import amg_amd as A
import oracle
from amg_amd._native import SSS_SMTR, dptr, iptr
from conftest import device_mode_oracle_opts, build_hierarchy, oracle_solve, vec

pytestmark = pytest.mark.gpu


def _lib():
    return A.lib()


@pytest.fixture(scope="module")
def bus_h(bus_matrix, quiet):
    return build_hierarchy(bus_matrix, quiet)


@pytest.fixture(scope="module")
def p32_h(quiet):
    return build_hierarchy(A.generate(7, 32), quiet)


@pytest.fixture(scope="module")
def a27_h(quiet):
    return build_hierarchy(A.generate(27, 16), quiet)


def test_device_present():
    assert A.device_count() >= 1


# ---------------------------------------------------------------- SpMV family, bitwise
@pytest.fixture(params=["tile", "tile-sorted", "tile-unsorted", "wave", "lean"])
def row_path(request, monkeypatch):
    """Run a test with every storage format a level qualifies for (dictionary tiles where every
    block qualifies, else column-sorted tiles; SSS_HIP_FORMATS=full, since the exact smoother's
    own default is plain tiles), with the column-sorted tiles only (SSS_HIP_DICT=0), with the tiles
    staged in stored order (SSS_HIP_SORTED_TILES=0 too), with every matrix forced onto the
    wave-per-row kernels (SSS_HIP_WAVE_MIN=1), and with the exact smoother's default plain tiles
    (lean), so every row path is checked bitwise."""
    monkeypatch.setenv("SSS_HIP_FORMATS", "lean" if request.param == "lean" else "full")
    if request.param == "wave":
        monkeypatch.setenv("SSS_HIP_WAVE_MIN", "1")
    if request.param in ("tile-sorted", "tile-unsorted"):
        monkeypatch.setenv("SSS_HIP_DICT", "0")
    if request.param == "tile-unsorted":
        monkeypatch.setenv("SSS_HIP_SORTED_TILES", "0")
    return request.param


@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h"])
@pytest.mark.parametrize("op", ["mxy", "amxpy", "resid", "acc"])
def test_spmv_bitwise_all_levels(request, hname, op, row_path):
    H = request.getfixturevalue(hname)
    ora = oracle.load()
    rng = np.random.default_rng(7)
    for l in range(H.num_levels):
        mats = [("A", H.level(l).A)]
        if l < H.num_levels - 1:
            mats += [("P", H.level(l).P), ("R", H.level(l).R)]
        for name, M in mats:
            x = rng.standard_normal(M.num_cols)
            b = rng.standard_normal(M.num_rows)
            y0 = rng.standard_normal(M.num_rows)
            y_gpu, y_ref = y0.copy(), y0.copy()
            alpha = -1.0 if op in ("resid", "amxpy") else 1.0
            cap = 100 if op == "acc" else 0
            rc = _lib().sss_hip_host_spmv(A.SPMV[op], alpha, C.byref(M), dptr(x), dptr(b), dptr(y_gpu), cap)
            assert rc == 0
            if op == "mxy":
                ora.ora_mv_mxy(C.byref(M), dptr(x), dptr(y_ref))
            elif op == "amxpy":
                ora.ora_mv_amxpy(alpha, C.byref(M), dptr(x), dptr(y_ref), 0)
            elif op == "resid":
                y_ref[:] = b
                ora.ora_mv_amxpy(-1.0, C.byref(M), dptr(x), dptr(y_ref), 0)
            else:
                ora.ora_mv_acc(C.byref(M), dptr(x), dptr(y_ref), cap)
            assert np.array_equal(y_gpu.view(np.uint64), y_ref.view(np.uint64)), (hname, l, name, op)


def test_host_entry_cache_follows_matrix_contents():
    """The host-memory entry points keep the device form of their operator between calls (keyed by
    a content hash): repeated calls give the oracle's result, and a value changed in place is seen
    by the next call (no stale device copy)."""
    rng = np.random.default_rng(11)
    n = 5000
    lens = rng.integers(1, 30, n)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ci = rng.integers(0, n, rp[-1]).astype(np.int32)
    v = rng.standard_normal(rp[-1])
    M = A.NumpyCSR(rp, ci, v)
    ora = oracle.load()
    x = rng.standard_normal(n)
    _lib().sss_hip_host_cache_clear()
    for it in range(3):
        if it == 2:
            M.v[17] += 1.0   # in place: same pointers, new contents
        y_gpu, y_ref = np.zeros(n), np.zeros(n)
        assert _lib().sss_hip_host_spmv(A.SPMV["mxy"], 1.0, C.byref(M.mat), dptr(x), None, dptr(y_gpu), 0) == 0
        ora.ora_mv_mxy(C.byref(M.mat), dptr(x), dptr(y_ref))
        assert np.array_equal(y_gpu.view(np.uint64), y_ref.view(np.uint64)), it
    _lib().sss_hip_host_cache_clear()


def test_spmv_long_rows_bitwise():
    """Rows longer than the LDS tile (2048) take the wave-parallel product path."""
    n = 300
    rng = np.random.default_rng(3)
    lens = np.where(np.arange(n) % 37 == 0, 5000, rng.integers(0, 40, n))
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ci = rng.integers(0, n, rp[-1]).astype(np.int32)
    v = rng.standard_normal(rp[-1])
    M = A.NumpyCSR(rp, ci, v)
    x = rng.standard_normal(n)
    y_gpu, y_ref = np.zeros(n), np.zeros(n)
    assert _lib().sss_hip_host_spmv(A.SPMV["mxy"], 1.0, C.byref(M.mat), dptr(x), None, dptr(y_gpu), 0) == 0
    oracle.load().ora_mv_mxy(C.byref(M.mat), dptr(x), dptr(y_ref))
    assert np.array_equal(y_gpu.view(np.uint64), y_ref.view(np.uint64))


def _powerlaw_csr(n, banded, seed):
    """A G3_circuit-sized irregular CSR (BASELINE.json configs[3]; the SuiteSparse file is not in
    the container): heavy-tailed row lengths 1..~3000 plus a few rows longer than the LDS tile;
    banded = columns within +-60,000 of the row (the sorted-tile path), else uniform over all columns
    (sorted tiles refused: stored-order staging)."""
    rng = np.random.default_rng(seed)
    lens = np.minimum(1 + rng.zipf(1.8, n), 3000)
    lens[rng.integers(0, n, 8)] = 6000
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    rows = np.repeat(np.arange(n), lens)
    if banded:
        ci = np.clip(rows + rng.integers(-60000, 60001, rp[-1]), 0, n - 1)
    else:
        ci = rng.integers(0, n, rp[-1])
    v = rng.standard_normal(rp[-1])
    return A.NumpyCSR(rp.astype(np.int32), ci.astype(np.int32), v)


@pytest.mark.parametrize("banded", [True, False])
@pytest.mark.parametrize("op", ["mxy", "resid"])
def test_spmv_irregular_large_bitwise(banded, op, row_path):
    """Load-balance path at G3_circuit size (1,585,478 rows): every row sum bitwise the oracle's."""
    n = 1585478
    M = _powerlaw_csr(n, banded, 11)
    rng = np.random.default_rng(12)
    x = rng.standard_normal(n)
    b = rng.standard_normal(n)
    y_gpu = np.zeros(n)
    y_ref = b.copy() if op == "resid" else np.zeros(n)
    assert _lib().sss_hip_host_spmv(A.SPMV[op], -1.0 if op == "resid" else 1.0, C.byref(M.mat), dptr(x),
                                    dptr(b) if op == "resid" else None, dptr(y_gpu), 0) == 0
    if op == "resid":
        oracle.load().ora_mv_amxpy(-1.0, C.byref(M.mat), dptr(x), dptr(y_ref), 0)
    else:
        oracle.load().ora_mv_mxy(C.byref(M.mat), dptr(x), dptr(y_ref))
    assert np.array_equal(y_gpu.view(np.uint64), y_ref.view(np.uint64))


def test_spmv_empty_rows():
    rp = np.array([0, 0, 2, 2, 3, 3], np.int32)
    ci = np.array([0, 4, 1], np.int32)
    v = np.array([1.5, -2.0, 3.0])
    M = A.NumpyCSR(rp, ci, v)
    x = np.arange(5, dtype=np.float64) + 1
    y = np.full(5, 7.0)
    assert _lib().sss_hip_host_spmv(A.SPMV["mxy"], 1.0, C.byref(M.mat), dptr(x), None, dptr(y), 0) == 0
    assert np.array_equal(y, [0.0, 1.5 - 10.0, 0.0, 6.0, 0.0])


# ---------------------------------------------------------------- smoother, bitwise
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


@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h"])
@pytest.mark.parametrize("post", [False, True])
def test_gscf_bitwise_all_levels(request, hname, post, row_path):
    H = request.getfixturevalue(hname)
    ora = oracle.load()
    rng = np.random.default_rng(11)
    for l in range(H.num_levels - 1):
        L = H.level(l)
        n = L.A.num_rows
        b = rng.standard_normal(n)
        x0 = rng.standard_normal(n)
        xg, xr = x0.copy(), x0.copy()
        sg = _smtr(L.A, b, xg, L.cfmark.d, 2, post)
        sr = _smtr(L.A, b, xr, L.cfmark.d, 2, post)
        assert _lib().sss_hip_host_smooth(C.byref(sg), int(post)) == 0
        (ora.ora_smoother_post if post else ora.ora_smoother_pre)(C.byref(sr))
        assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64)), (hname, l)


def test_gscf_missing_diagonal_stale_d():
    """Rows without a diagonal reuse the previous divisor (Solve/SSS_smooth.c:30,46)."""
    rng = np.random.default_rng(5)
    n = 40
    rows = []
    for i in range(n):
        cols = sorted(set(rng.integers(0, n, 4).tolist()) | ({i} if i % 7 else set()))
        rows.append(cols)
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
    ci = np.array([c for r in rows for c in r], np.int32)
    v = np.array([4.0 + i if c == i else -0.3 for i, r in enumerate(rows) for c in r])
    M = A.NumpyCSR(rp, ci, v)
    mark = np.array([(i * 5) % 3 == 0 for i in range(n)], np.int32)
    b = rng.standard_normal(n)
    x0 = rng.standard_normal(n)
    xg, xr = x0.copy(), x0.copy()
    sg = _smtr(M.mat, b, xg, iptr(mark), 3, False)
    sr = _smtr(M.mat, b, xr, iptr(mark), 3, False)
    assert _lib().sss_hip_host_smooth(C.byref(sg), 0) == 0
    oracle.load().ora_smoother_pre(C.byref(sr))
    assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64))


@pytest.mark.parametrize("hname", ["bus_h", "p32_h"])
def test_cf_jacobi_bitwise(request, hname, row_path):
    H = request.getfixturevalue(hname)
    ora = oracle.load()
    rng = np.random.default_rng(2)
    for l in range(H.num_levels - 1):
        L = H.level(l)
        n = L.A.num_rows
        b = rng.standard_normal(n)
        x0 = rng.standard_normal(n)
        xg, xr = x0.copy(), x0.copy()
        sg = _smtr(L.A, b, xg, L.cfmark.d, 2, False, smoother=1)
        assert _lib().sss_hip_host_smooth(C.byref(sg), 0) == 0
        ora.ora_cf_jacobi(dptr(xr), C.byref(L.A), dptr(b), 2, L.cfmark.d)
        assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64)), (hname, l)


# ---------------------------------------------------------------- coarse solve
def _cg_form(mp, step):
    """persist: the whole CG loop in one launch (k_cg_persist, the default for n <= 4096); reg: the
    register step and the SpMV as two kernels per iteration; lds: the LDS-chunked step."""
    mp.setenv("SSS_HIP_CG_REG", "0" if step == "lds" else "1")
    mp.setenv("SSS_HIP_CG_PERSIST", "1" if step == "persist" else "0")


@pytest.mark.parametrize("step", ["persist", "reg", "lds"])
@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h"])
def test_coarse_krylov_matches_oracle(request, hname, step, monkeypatch):
    """Every CG form (one launch; register-resident step, n <= 4096; LDS-chunked, SSS_HIP_CG_REG=0)."""
    _cg_form(monkeypatch, step)
    H = request.getfixturevalue(hname)
    Lc = H.level(H.num_levels - 1)
    n = Lc.A.num_rows
    rng = np.random.default_rng(9)
    b = rng.standard_normal(n)
    xg, xr = np.zeros(n), np.zeros(n)
    assert _lib().sss_hip_host_coarse_solve(C.byref(Lc.A), C.byref(vec(b)), C.byref(vec(xg)), 1e-7, 0, 0) == 0
    oracle.load().ora_coarest_solve(C.byref(Lc.A), C.byref(vec(b)), C.byref(vec(xr)), 1e-7,
                                    C.byref(oracle.opts()))
    assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64))


@pytest.mark.parametrize("step", ["persist", "reg", "lds"])
@pytest.mark.parametrize("lo,hi", [(1025, 4096), (4097, 40000)])
def test_coarse_krylov_larger_grids(p32_h, lo, hi, step, monkeypatch):
    """A finer level as the 'coarsest' matrix: several entries per thread in the register step
    (1025..4096 rows), the LDS-chunked step past 4096 rows and its multi-chunk sequential sums."""
    _cg_form(monkeypatch, step)
    L = next(p32_h.level(l) for l in range(p32_h.num_levels) if lo <= p32_h.level(l).A.num_rows <= hi)
    n = L.A.num_rows
    b = np.random.default_rng(4).standard_normal(n)
    xg, xr = np.zeros(n), np.zeros(n)
    assert _lib().sss_hip_host_coarse_solve(C.byref(L.A), C.byref(vec(b)), C.byref(vec(xg)), 1e-7, 0, 0) == 0
    oracle.load().ora_coarest_solve(C.byref(L.A), C.byref(vec(b)), C.byref(vec(xr)), 1e-7,
                                    C.byref(oracle.opts()))
    assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64))


@pytest.mark.parametrize("step", ["persist", "reg"])
@pytest.mark.parametrize("n", [1, 2, 17, 1024, 4095, 4096, 4097])
def test_coarse_krylov_step_sizes(n, step, monkeypatch):
    """The register CG step and the one-launch CG at their size edges (one entry per thread up to
    four; one row per worker wave; 4097 rows take the LDS-chunked step): a shifted 1-D Laplacian with
    a random right-hand side."""
    _cg_form(monkeypatch, step)
    import scipy.sparse as sp
    M = sp.diags([-np.ones(n - 1), np.full(n, 2.05), -np.ones(n - 1)], [-1, 0, 1], format="csr") \
        if n > 1 else sp.csr_matrix(np.array([[2.05]]))
    M.sort_indices()
    hold = A.NumpyCSR(M.indptr, M.indices, M.data)
    b = np.random.default_rng(n).standard_normal(n)
    xg, xr = np.zeros(n), np.zeros(n)
    assert _lib().sss_hip_host_coarse_solve(C.byref(hold.mat), C.byref(vec(b)), C.byref(vec(xg)), 1e-7, 0, 0) == 0
    oracle.load().ora_coarest_solve(C.byref(hold.mat), C.byref(vec(b)), C.byref(vec(xr)), 1e-7,
                                    C.byref(oracle.opts()))
    assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64))


@pytest.mark.parametrize("step", ["persist", "reg"])
def test_coarse_krylov_long_rows(step, monkeypatch):
    """Rows longer than one tile (2,048 entries) -- the double-buffered block-row chain -- in the
    coarse CG / GMRES SpMVs: a 2,600-row matrix whose first 24 rows and columns are dense."""
    import scipy.sparse as sp
    n, k = 2600, 24
    rng = np.random.default_rng(12)
    S = sp.random(n, n, density=6.0 / n, random_state=rng, format="csr")
    D = sp.lil_matrix((n, n))
    D[:k, :] = rng.uniform(-1.0, 1.0, (k, n))
    M = S + S.T + D + D.T
    M = (M + sp.diags(np.asarray(abs(M).sum(axis=1)).ravel() + 1.0)).tocsr()
    M.sort_indices()
    assert np.diff(M.indptr).max() > 2048
    _cg_form(monkeypatch, step)
    hold = A.NumpyCSR(M.indptr, M.indices, M.data)
    b = rng.standard_normal(n)
    xg, xr = np.zeros(n), np.zeros(n)
    assert _lib().sss_hip_host_coarse_solve(C.byref(hold.mat), C.byref(vec(b)), C.byref(vec(xg)), 1e-7, 0, 0) == 0
    oracle.load().ora_coarest_solve(C.byref(hold.mat), C.byref(vec(b)), C.byref(vec(xr)), 1e-7,
                                    C.byref(oracle.opts()))
    assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64))


@pytest.mark.parametrize("step", ["persist", "reg"])
@pytest.mark.parametrize("cap", [0, 40])
def test_coarse_krylov_row_cap(bus_h, cap, step, monkeypatch):
    """The as-shipped <<<64,64>>> row cap (rows >= cap untouched by the coarse SpMVs)."""
    _cg_form(monkeypatch, step)
    Lc = bus_h.level(bus_h.num_levels - 1)
    n = Lc.A.num_rows
    b = np.linspace(-1.0, 2.0, n)
    xg, xr = np.zeros(n), np.zeros(n)
    assert _lib().sss_hip_host_coarse_solve(C.byref(Lc.A), C.byref(vec(b)), C.byref(vec(xg)), 1e-7, 0, cap) == 0
    oracle.load().ora_coarest_solve(C.byref(Lc.A), C.byref(vec(b)), C.byref(vec(xr)), 1e-7,
                                    C.byref(oracle.opts(row_cap=cap)))
    assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64))


def test_coarse_krylov_persist_stall_is_reported(bus_h, monkeypatch):
    """A stalled one-launch CG (SSS_HIP_CG_SPIN=-1: every bounded wait gives up at once) leaves the
    launch -- every workgroup reaches its exit -- and the coarse solve reports the error instead of
    returning the garbage iterate; the next launch (fresh tags, stall word cleared) solves bitwise."""
    _cg_form(monkeypatch, "persist")
    Lc = bus_h.level(bus_h.num_levels - 1)
    n = Lc.A.num_rows
    b = np.random.default_rng(21).standard_normal(n)
    xg, xr = np.zeros(n), np.zeros(n)
    monkeypatch.setenv("SSS_HIP_CG_SPIN", "-1")
    assert _lib().sss_hip_host_coarse_solve(C.byref(Lc.A), C.byref(vec(b)), C.byref(vec(xg)), 1e-7, 0, 0) != 0
    monkeypatch.delenv("SSS_HIP_CG_SPIN")
    xg[:] = 0.0
    assert _lib().sss_hip_host_coarse_solve(C.byref(Lc.A), C.byref(vec(b)), C.byref(vec(xg)), 1e-7, 0, 0) == 0
    oracle.load().ora_coarest_solve(C.byref(Lc.A), C.byref(vec(b)), C.byref(vec(xr)), 1e-7,
                                    C.byref(oracle.opts()))
    assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64))


def test_coarse_direct_solves(p32_h):
    Lc = p32_h.level(p32_h.num_levels - 1)
    n = Lc.A.num_rows
    rng = np.random.default_rng(1)
    b = rng.standard_normal(n)
    x = np.zeros(n)
    assert _lib().sss_hip_host_coarse_solve(C.byref(Lc.A), C.byref(vec(b)), C.byref(vec(x)), 1e-7, 1, 0) == 0
    rp, ci, v = A.csr_arrays(Lc.A)
    Ax = np.zeros(n)
    for i in range(n):
        Ax[i] = np.dot(v[rp[i]:rp[i + 1]], x[ci[rp[i]:rp[i + 1]]])
    assert np.linalg.norm(Ax - b) <= 1e-10 * np.linalg.norm(b)


# ---------------------------------------------------------------- whole solve
def _gpu_history(H, smoother="exact", coarse="krylov", row_cap=0, max_it=100, relabel=None, graph=None, inner=None,
                 inner_from=None):
    n = H.level(0).A.num_rows
    D = A.DeviceHierarchy(H, smoother=smoother, coarse=coarse, row_cap=row_cap, relabel=relabel, graph=graph,
                          inner=inner, inner_from=inner_from)
    b = np.ones(n)
    D.upload(0, "b", b)
    D.upload(0, "x", np.ones(n))
    sumb = np.sqrt(np.dot(b, b))
    rel = []
    for _ in range(max_it):
        D.cycle()
        rel.append(D.residual_norm() / sumb)
        if rel[-1] < H.pars.tol:
            break
    x = D.download(0, "x")
    D.close()
    return np.array(rel), x


def _oracle_history(H, **kw):
    n = H.level(0).A.num_rows
    b, x = np.ones(n), np.ones(n)
    rtn, rel, _ = oracle_solve(H, b, x, **kw)
    return rel, x


@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h"])
def test_solve_parity_mode(request, hname, row_path):
    H = request.getfixturevalue(hname)
    rel_r, x_r = _oracle_history(H)
    rel_g, x_g = _gpu_history(H)
    assert len(rel_g) == len(rel_r)
    # x is bitwise identical; only the level-0 norm is reduced in tree order on the GPU
    assert np.array_equal(x_g.view(np.uint64), x_r.view(np.uint64))
    assert np.allclose(rel_g, rel_r, rtol=1e-13, atol=0)


@pytest.mark.parametrize("hname", ["p32_h", "a27_h"])
def test_solve_direct_coarse(request, hname):
    H = request.getfixturevalue(hname)
    rel_r, x_r = _oracle_history(H)
    rel_g, x_g = _gpu_history(H, coarse="direct")
    assert len(rel_g) == len(rel_r)
    assert np.allclose(rel_g, rel_r, rtol=1e-6, atol=0)
    assert np.linalg.norm(x_g - x_r) <= 1e-6 * np.linalg.norm(x_r)


def _mask(inner_from):
    """oracle inner_mask for 'two-stage on levels >= inner_from'"""
    return ~((1 << inner_from) - 1)


@pytest.mark.parametrize("inner,inner_from", [(0, 2), (1, 1), (1, 2)])
def test_solve_hybrid_jacobi_converges(p32_h, inner, inner_from):
    kw = device_mode_oracle_opts(p32_h, smoother="hybrid", coarse="direct", inner=inner, inner_from=inner_from)
    assert kw["inner_mask"] & ~_mask(inner_from) == 0   # 7-pt level 0 is chain-free: exact there
    rel_o, x_o = _oracle_history(p32_h, **kw)
    rel_g, x_g = _gpu_history(p32_h, smoother="hybrid", coarse="direct", inner=inner, inner_from=inner_from)
    assert len(rel_g) == len(rel_o)
    assert np.allclose(rel_g, rel_o, rtol=1e-6)
    rel_ref, _ = _oracle_history(p32_h)
    assert len(rel_g) <= len(rel_ref) + 2


@pytest.mark.parametrize("hname", ["p32_h", "a27_h"])
@pytest.mark.parametrize("inner", [0, 1])
def test_w_cycle_throughput_matches_oracle(request, hname, inner):
    """cycle_type = 2 in throughput mode: a level re-descended after its post-smoother (the W-cycle's
    second visit, Solve/SSS_cycle.cu:959-966) starts its pre-smoother from that iterate, not from
    the zero the first descent left -- so the zero-iterate first pass (t = b, no matrix read) must
    not be taken there.  The history follows the oracle's W-cycle in the same per-level
    configuration."""
    H = request.getfixturevalue(hname)
    H.mg.pars.cycle_type = 2
    try:
        kw = device_mode_oracle_opts(H, smoother="hybrid", coarse="direct", inner=inner, inner_from=1)
        rel_o, x_o = _oracle_history(H, **kw)
        rel_g, x_g = _gpu_history(H, smoother="hybrid", coarse="direct", inner=inner, inner_from=1)
    finally:
        H.mg.pars.cycle_type = 1
    assert len(rel_g) == len(rel_o)
    assert np.allclose(rel_g, rel_o, rtol=1e-6)
    assert np.linalg.norm(x_g - x_o) <= 1e-8 * np.linalg.norm(x_o)


@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h"])
@pytest.mark.parametrize("smoother,coarse", [("exact", "krylov"), ("hybrid", "direct"), ("jacobi", "direct")])
def test_relabel_is_bitwise_neutral(request, hname, smoother, coarse):
    """The device F|C renumbering (sss_hier.hip relabel_csr) changes only labels: the iterates with
    it on/off (and with graph replay on/off) are bitwise identical."""
    H = request.getfixturevalue(hname)
    rel0, x0 = _gpu_history(H, smoother, coarse, max_it=12, relabel=0, graph=0)
    rel1, x1 = _gpu_history(H, smoother, coarse, max_it=12, relabel=1, graph=1)
    assert len(rel0) == len(rel1)
    assert np.array_equal(x0.view(np.uint64), x1.view(np.uint64))
    assert np.allclose(rel0, rel1, rtol=1e-13, atol=0)


@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h"])
@pytest.mark.parametrize("smoother,inner", [("exact", 0), ("jacobi", 0), ("jacobi", 1), ("jacobi", 2)])
def test_relabeled_level_smoothers_bitwise(request, hname, smoother, inner, row_path):
    """Per level, through the relabeled mirror: upload (b, x) in the caller's labels, run the device
    pre/post smoother (GS-CF, C/F-Jacobi or two-stage GS-CF), download, compare bitwise with the
    oracle on the original labels."""
    H = request.getfixturevalue(hname)
    ora = oracle.load()
    D = A.DeviceHierarchy(H, smoother=smoother, coarse="direct", relabel=1, inner=inner, inner_from=0)
    rng = np.random.default_rng(23)
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
                assert np.array_equal(D.download(l, "b").view(np.uint64), b.view(np.uint64))
                xr = x0.copy()
                sweeps = H.pars.post_iter if post else H.pars.pre_iter
                if smoother == "jacobi" and inner > 0:
                    ora.ora_cf_twostage(dptr(xr), C.byref(L.A), dptr(b), sweeps, L.cfmark.d, inner)
                elif smoother == "jacobi":
                    ora.ora_cf_jacobi(dptr(xr), C.byref(L.A), dptr(b), sweeps, L.cfmark.d)
                else:
                    sr = _smtr(L.A, b, xr, L.cfmark.d, sweeps, post)
                    (ora.ora_smoother_post if post else ora.ora_smoother_pre)(C.byref(sr))
                assert np.array_equal(xg.view(np.uint64), xr.view(np.uint64)), (hname, l, post)
    finally:
        D.close()


@pytest.mark.parametrize("hname", ["bus_h", "p32_h", "a27_h"])
@pytest.mark.parametrize("inner,inner_from", [(0, 2), (1, 1), (1, 2), (2, 2)])
def test_solve_hybrid_krylov_bitwise(request, hname, inner, inner_from, row_path):
    """Throughput smoothers with the reference coarse solver: x bitwise equal to the oracle's."""
    H = request.getfixturevalue(hname)
    kw = device_mode_oracle_opts(H, smoother="hybrid", coarse="krylov", inner=inner, inner_from=inner_from)
    rel_r, x_r = _oracle_history(H, **kw)
    rel_g, x_g = _gpu_history(H, smoother="hybrid", coarse="krylov", inner=inner, inner_from=inner_from)
    assert len(rel_g) == len(rel_r)
    assert np.array_equal(x_g.view(np.uint64), x_r.view(np.uint64))
    assert np.allclose(rel_g, rel_r, rtol=1e-13, atol=0)


@pytest.mark.parametrize("knob", ["SSS_HIP_FUSE_RESID", "SSS_HIP_DEAD_PROLONG", "SSS_HIP_TILE_DIAG", "SSS_HIP_PEND_F",
                                  "SSS_HIP_ZERO_FIRST", "SSS_HIP_INJECT", "SSS_HIP_ELL_BASE"])
@pytest.mark.parametrize("smoother,coarse", [("exact", "krylov"), ("hybrid", "direct")])
def test_fused_residual_bitwise(p32_h, smoother, coarse, knob, monkeypatch):
    """Level 0 of 7-pt Poisson is red-black.  SSS_HIP_FUSE_RESID: the last C pass of each smoother
    call also writes the C rows of r = b - A x (ResidFuse).  SSS_HIP_DEAD_PROLONG: the prolongation
    skips the F rows, which the post-smoother's first (depth-1) F pass overwrites from C values
    only.  SSS_HIP_TILE_DIAG: tile passes divide by the diagonal staged from the sorted tile
    instead of reading the divisor stream.  SSS_HIP_PEND_F: the outer residual's F half also
    computes the next cycle's first F pass, which the cycle then skips.  SSS_HIP_ZERO_FIRST: the
    first C/F-Jacobi or two-stage pass of a coarse level's pre-smoother (x just zeroed) reduces to
    t = b without reading the matrix.  SSS_HIP_INJECT: that C-row prolongation, whose rows are each
    one stored 1.0, reads only their columns (prolong_inject) instead of the tiles.
    SSS_HIP_ELL_BASE: the restriction as a dictionary ELL whose offsets are taken against each row's
    first column (DevCSR::dv_ell_base) instead of the column ELL.  With each
    on/off: x, the in-cycle residual wp and the
    outer residual norm are bitwise
    identical over several cycles."""
    n = p32_h.level(0).A.num_rows
    out = []
    for fuse in ("1", "0"):
        monkeypatch.setenv(knob, fuse)
        D = A.DeviceHierarchy(p32_h, smoother=smoother, coarse=coarse)
        D.upload(0, "b", np.ones(n))
        D.upload(0, "x", np.ones(n))
        norms = []
        for _ in range(4):
            D.cycle()
            norms.append(D.residual_norm())
        out.append((np.array(norms), D.download(0, "x"), D.download(0, "wp")))
        D.close()
    (n1, x1, w1), (n0, x0, w0) = out
    assert np.array_equal(n1.view(np.uint64), n0.view(np.uint64))
    assert np.array_equal(x1.view(np.uint64), x0.view(np.uint64))
    assert np.array_equal(w1.view(np.uint64), w0.view(np.uint64))


@pytest.mark.parametrize("hname", ["p32_h", "a27_h"])
@pytest.mark.parametrize("smoother,inner", [("hybrid", 0), ("hybrid", 1), ("jacobi", 2)])
def test_nocopy_jacobi_bitwise(request, hname, smoother, inner, monkeypatch):
    """C/F-Jacobi and two-stage passes writing into a second x vector and reading each class from
    where its current values live (SmootherPlan::x2) give the iterates of the copy-per-pass form."""
    H = request.getfixturevalue(hname)
    xs = []
    for nc in ("1", "0"):
        monkeypatch.setenv("SSS_HIP_NOCOPY", nc)
        rel, x = _gpu_history(H, smoother, "direct", max_it=6, inner=inner, inner_from=1)
        xs.append((rel, x))
    assert np.array_equal(xs[0][1].view(np.uint64), xs[1][1].view(np.uint64))
    assert np.array_equal(xs[0][0].view(np.uint64), xs[1][0].view(np.uint64))


def test_solve_bus_known_answer(bus_h):
    """GPU history equals the reference's printed table."""
    expect = [2.907170e+00, 4.389125e-01, 1.321964e-01, 4.453643e-02, 1.213532e-02, 3.537244e-03, 1.358532e-03,
              3.614966e-04, 1.381984e-04, 2.328166e-05, 9.120090e-06, 2.602226e-06, 8.230269e-07]
    rel, _ = _gpu_history(bus_h)
    assert ["%.6e" % r for r in rel] == ["%.6e" % r for r in expect]


@pytest.mark.parametrize("overlap", ["1", "0"])
def test_drop_in_solver_amg(bus_matrix, capfd, overlap, monkeypatch):
    """SSS_solver_amg through the C ABI prints the reference's table and fills the caller's x --
    with the HBM mirror built while the setup runs (default) and in the reference's sequence
    (setup, then the mirror at the first solve: SSS_HIP_OVERLAP_SETUP=0)."""
    monkeypatch.setenv("SSS_HIP_OVERLAP_SETUP", overlap)
    n = bus_matrix.num_rows
    b, x = np.ones(n), np.ones(n)
    pars = A.default_pars()
    rtn = _lib().SSS_solver_amg(C.byref(bus_matrix), C.byref(vec(x)), C.byref(vec(b)), C.byref(pars))
    C.CDLL(None).fflush(None)
    out = capfd.readouterr().out
    assert rtn.nits == 13
    assert "    13 |  8.230269e-07   |  2.776420e-05  |     0.3163" in out
    rel_r, x_r = _oracle_history(build_hierarchy(bus_matrix, type(
        "Q", (), {"__enter__": lambda s: None, "__exit__": lambda s, *a: None})))
    assert np.linalg.norm(x - x_r) <= 1e-10 * np.linalg.norm(x_r)


def test_reference_main_dropin():
    """The reference's unmodified SSS_main.c linked against libsss_amg.so."""
    import subprocess
    from pathlib import Path
    from conftest import BUS_MTX, GOLDEN
    exe = Path(oracle.__file__).resolve().parent / "_ref" / "amg_dropin"
    if not exe.exists():
        pytest.skip("built only where the reference tree was present")
    r = subprocess.run([str(exe), str(BUS_MTX)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    import json
    g = json.loads((GOLDEN / "golden.json").read_text())["survey"]["bus_history"]
    rows = [l.split("|") for l in r.stdout.splitlines() if l[:6].strip().isdigit() and "|" in l]
    assert ["%s" % c[1].strip() for c in rows] == g["relres"]
    assert "AMG iterations: 13" in r.stdout
