"""Synthetic operators for the workloads BASELINE.json names whose files are not in the container.

circuit(n): the G3_circuit stand-in (BASELINE.json configs[3], SuiteSparse G3_circuit: 1,585,478
rows, ~7.66M nonzeros, SPD, a circuit-simulation graph).  The SuiteSparse file cannot be fetched
here, so this builds an operator of the same size and kind: a weighted graph Laplacian plus a small
diagonal shift (symmetric, diagonally dominant, positive diagonal and non-positive off-diagonals --
an M-matrix, the class classical RS coarsening, Setup/SSS_coarsen.c, is built for) over

- a 2-D grid of conductors with ~20% of the links removed (ragged rows of 1..4 neighbours);
- local "wires": one per ~10 nodes, to a node a Gaussian distance (sigma 4 grid cells) away;
- "power nets": a few hub nodes, each tied to a heavy-tailed (Pareto) number of nodes -- up to
  several thousand -- within +-50,000 labels (rows longer than the LDS tile: the load-balance path);

conductances are log-normal.  Deterministic in (n, seed).  Rows are column-sorted CSR.
"""
from __future__ import annotations

import numpy as np

G3_CIRCUIT_ROWS = 1585478


def circuit_coo(n: int, seed: int = 7):
    rng = np.random.default_rng(seed)
    side = int(np.ceil(np.sqrt(n)))
    i = np.arange(n, dtype=np.int64)
    col = i % side
    src, dst = [], []
    right = (col + 1 < side) & (i + 1 < n)
    down = i + side < n
    for m, off in ((right, 1), (down, side)):
        keep = m & (rng.random(n) < 0.8)
        src.append(i[keep])
        dst.append(i[keep] + off)
    nw = n // 10   # local wires
    a = rng.integers(0, n, nw)
    dx, dy = np.rint(rng.normal(0.0, 4.0, (2, nw))).astype(np.int64)
    b = np.clip(a + dx + dy * side, 0, n - 1)
    src.append(a)
    dst.append(b)
    nh = max(1, n // 50000)   # power nets
    hubs = rng.integers(0, n, nh)
    deg = np.minimum(200 * (1.0 + rng.pareto(0.8, nh)), 6000).astype(np.int64)
    for h, d in zip(hubs, deg):
        t = np.clip(h + rng.integers(-50000, 50001, int(d)), 0, n - 1)
        src.append(np.full(len(t), h, dtype=np.int64))
        dst.append(t)
    s = np.concatenate(src)
    t = np.concatenate(dst)
    keep = s != t
    s, t = s[keep], t[keep]
    w = np.exp(rng.normal(0.0, 1.0, len(s)))
    return s, t, w


def circuit(n: int = G3_CIRCUIT_ROWS, seed: int = 7, shift: float = 1e-2):
    """(row_ptr, col_idx, val) of the stand-in operator, int32/int32/float64."""
    import scipy.sparse as sp
    s, t, w = circuit_coo(n, seed)
    # parallel links summed once in the upper triangle, then mirrored: exactly symmetric
    U = sp.coo_matrix((w, (np.minimum(s, t), np.maximum(s, t))), shape=(n, n)).tocsr()
    U.sum_duplicates()
    W = (U + U.T).tocsr()
    deg = np.asarray(W.sum(axis=1)).ravel()
    A = (sp.diags(deg + shift * max(deg.mean(), 1.0)) - W).tocsr()
    A.sum_duplicates()
    A.sort_indices()
    return A.indptr.astype(np.int32), A.indices.astype(np.int32), A.data.astype(np.float64)


def circuit_csr(n: int = G3_CIRCUIT_ROWS, seed: int = 7):
    """The stand-in as an amg_amd.NumpyCSR (its .mat is an SSS_MAT view)."""
    from ._native import NumpyCSR
    return NumpyCSR(*circuit(n, seed))
