"""The G3_circuit stand-in generator (amg_amd/workloads.py; BASELINE.json configs[3]) on CPU:
deterministic, symmetric M-matrix, G3_circuit's size and a heavy tail of rows longer than the LDS
tile, and the oracle's reference-semantics solve converges on it.  (The SuiteSparse G3_circuit file
is not in the container: the operator is synthetic, so its iteration counts are parity unpinned
against the reference -- the GPU tests pin the device against the oracle on it.)"""
from __future__ import annotations

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import build_hierarchy, oracle_solve, quiet_ctx
from amg_amd import workloads as W


def _mat(n, seed=7):
    rp, ci, v = W.circuit(n, seed)
    return sp.csr_matrix((v, ci, rp), shape=(n, n))


def test_circuit_deterministic_spd_structure():
    A1, A2 = _mat(50000), _mat(50000)
    assert (A1 != A2).nnz == 0
    assert abs(A1 - A1.T).max() == 0.0
    d = A1.diagonal()
    off = A1 - sp.diags(d)
    assert (d > 0).all() and off.max() <= 0.0
    assert (d > -np.asarray(off.sum(axis=1)).ravel()).all()   # strictly diagonally dominant
    assert (np.diff(A1.indptr) > 0).all()
    for r in (0, 17, 49999):   # column-sorted rows
        cols = A1.indices[A1.indptr[r]:A1.indptr[r + 1]]
        assert (np.diff(cols) > 0).all()


def test_circuit_full_size_shape():
    rp, ci, v = W.circuit(W.G3_CIRCUIT_ROWS)
    lens = np.diff(rp)
    assert len(lens) == 1585478
    assert 6_500_000 < rp[-1] < 8_000_000      # G3_circuit: 7,660,826
    assert (lens > 2048).sum() >= 1             # rows longer than one LDS tile (kTileEntries)
    assert lens.min() >= 1


def test_circuit_oracle_converges():
    M = W.circuit_csr(50000)
    H = build_hierarchy(M.mat, quiet_ctx)
    n = H.level(0).A.num_rows
    rtn, rel, _ = oracle_solve(H, np.ones(n), np.ones(n))
    assert H.num_levels >= 4
    assert rel[-1] < H.pars.tol and len(rel) < 40


# ---- bench.py --mtx (BASELINE.json configs[0] nos5 / configs[3] G3_circuit when the files are supplied)
def test_bench_mtx_reads_like_the_reference(tmp_path):
    """bench.py --mtx goes through SSS_mat_read (the reference's ingest; tests/test_ref_units.py pins
    that reader to the compiled reference one): on 1138_bus the matrix it loads is the reader's CSR,
    and the workload is named after the file."""
    import ctypes as C
    import sys
    from conftest import BUS_MTX, ROOT
    sys.path.insert(0, str(ROOT))
    import amg_amd as A
    import bench
    M = bench.load_mtx(A, BUS_MTX)
    R = A.read_mtx(BUS_MTX)
    try:
        assert (M.num_rows, M.num_cols, M.num_nnzs) == (1138, 1138, 4054)
        n, z = M.num_rows, M.num_nnzs
        for f, k in (("row_ptr", n + 1), ("col_idx", z), ("val", z)):
            a = np.ctypeslib.as_array(getattr(M, f), shape=(k,))
            b = np.ctypeslib.as_array(getattr(R, f), shape=(k,))
            assert np.array_equal(a, b), f
    finally:
        A.lib().SSS_mat_destroy(C.byref(M))
        A.lib().SSS_mat_destroy(C.byref(R))

    class Args:
        n, stencil = None, 7
    assert bench.workload_name(Args, False, BUS_MTX) == "mtx_1138_bus"


def test_bench_mtx_cli(tmp_path):
    """The --mtx flag on the command line: the rank probe names the file's workload; a missing file
    and a multi-rank request fail before anything touches the GPU."""
    import json
    import subprocess
    import sys
    from conftest import BUS_MTX, ROOT
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--probe-ranks", "--mtx", str(BUS_MTX)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip())["workload"] == "mtx_1138_bus"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--mtx", str(tmp_path / "nos5.mtx")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "no such file" in r.stderr
