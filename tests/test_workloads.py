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
