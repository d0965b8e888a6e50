"""Binary hierarchy file (SSS_amg_save / SSS_amg_load, amg_amd/host/sss_hierio.c; SURVEY.md §8f
row 2).  CPU: a loaded hierarchy is field-for-field the one SSS_amg_setup built, the oracle's
solve on it is bitwise the same, and damaged files are refused."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import amg_amd as A
from conftest import build_hierarchy, oracle_solve


def _csr(M):
    rp, ci, v = A.csr_arrays(M)
    return rp.copy(), ci.copy(), v.copy(), (M.num_rows, M.num_cols, M.num_nnzs)


def _same(M1, M2):
    a, b = _csr(M1), _csr(M2)
    assert a[3] == b[3]
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert np.array_equal(a[2].view(np.uint64), b[2].view(np.uint64))


@pytest.mark.parametrize("kind,n", [(7, 16), (27, 8), ("bus", 0)])
def test_save_load_roundtrip(tmp_path, quiet, bus_matrix, kind, n):
    M = bus_matrix if kind == "bus" else A.generate(kind, n)
    H = build_hierarchy(M, quiet)
    path = tmp_path / "h.sssamg"
    H.save(path)
    G = A.Hierarchy.load(path)
    assert G.num_levels == H.num_levels
    assert bytes(G.mg.pars) == bytes(H.mg.pars)
    for l in range(H.num_levels):
        _same(H.level(l).A, G.level(l).A)
        if l + 1 < H.num_levels:
            _same(H.level(l).P, G.level(l).P)
            _same(H.level(l).R, G.level(l).R)
            m = H.level(l).A.num_rows
            c1 = np.ctypeslib.as_array(H.level(l).cfmark.d, shape=(m,))
            c2 = np.ctypeslib.as_array(G.level(l).cfmark.d, shape=(m,))
            assert np.array_equal(c1, c2)
    N = H.level(0).A.num_rows
    x1, x2 = np.ones(N), np.ones(N)
    r1, rel1, _ = oracle_solve(H, np.ones(N), x1)
    r2, rel2, _ = oracle_solve(G, np.ones(N), x2)
    assert r1.nits == r2.nits
    assert np.array_equal(rel1, rel2)
    assert np.array_equal(x1.view(np.uint64), x2.view(np.uint64))
    G.close()


def test_load_refuses_damaged_files(tmp_path, quiet):
    H = build_hierarchy(A.generate(7, 8), quiet)
    path = tmp_path / "h.sssamg"
    H.save(path)
    raw = path.read_bytes()
    bad = tmp_path / "bad"
    for blob in (b"NOTAHIER" + raw[8:], raw[: len(raw) // 2], b""):
        bad.write_bytes(blob)
        with pytest.raises(OSError):
            A.Hierarchy.load(bad)
    with pytest.raises(OSError):
        A.Hierarchy.load(tmp_path / "missing")
