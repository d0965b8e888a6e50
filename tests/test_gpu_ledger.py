"""GPU: the stored-format byte ledger behind bench.py's `vcycle_stored` (sss_hip_cycle_bytes).

The ledger walks one outer iteration into a discarded stream capture: it must not change the
iterates or the engine's pending-pass state, and its per-level bytes must be consistent with the
level's stored formats (every smoothed level moves at least its matrix once and at most a few
times per smoother sweep)."""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

pytestmark = pytest.mark.gpu


def _cycles(D, n, k, ledger_every=False):
    D.upload(0, "b", np.ones(n))
    D.upload(0, "x", np.ones(n))
    out = []
    for _ in range(k):
        if ledger_every:
            D.cycle_bytes()
        D.cycle()
        out.append(D.residual_norm())
    return D.download(0, "x"), out


@pytest.mark.parametrize("kind,n,mode", [(7, 32, "throughput"), (27, 20, "throughput"), (7, 24, "parity")])
def test_cycle_bytes_no_side_effects_and_bounds(kind, n, mode):
    import amg_amd as A
    from conftest import build_hierarchy, quiet_ctx

    H = build_hierarchy(A.generate(kind, n), quiet_ctx)
    N = H.level(0).A.num_rows
    kw = dict(smoother="hybrid", coarse="direct", sum_order=1) if mode == "throughput" else \
        dict(smoother="exact", coarse="krylov", sum_order=0)
    D = A.DeviceHierarchy(H, device=0, **kw)
    x0, r0 = _cycles(D, N, 3)
    x1, r1 = _cycles(D, N, 3, ledger_every=True)   # the same cycles with the ledger walked before each
    assert np.array_equal(x0.view(np.uint64), x1.view(np.uint64))
    assert r0 == r1
    cb = D.cycle_bytes()
    nl = H.num_levels
    assert len(cb["levels"]) == nl
    assert cb["total"] == pytest.approx(sum(cb["levels"]) + cb["outer"] + cb["coarse"])
    tail = A.lib().sss_hip_tail_from(D.h)   # levels below a single-workgroup tail book into its first
    for l in range(nl - 1):
        if 0 < tail < l:
            assert cb["levels"][l] == 0.0
            continue
        info = D.level_info(l)
        stored = info.a_stream_bytes
        rows = H.level(l).A.num_rows
        # at least one pass over the matrix plus one vector; at most (sweeps + residual + 4) passes
        # over it with 20 row vectors each, plus R and P
        hi = 10 * stored + 200 * rows + 4 * 16 * H.level(l).P.num_nnzs
        if 0 < tail == l:
            hi = float("inf")
        assert 8 * rows < cb["levels"][l] <= hi, (l, cb["levels"][l], stored, rows)
    A0 = H.level(0).A
    # outer residual + norm: at least b, r and the gathered x; at most its CSR bytes + vectors
    assert 24 * N <= cb["outer"] <= 12 * A0.num_nnzs + 4 * (N + 1) + 48 * N
    if mode == "throughput" and tail <= 0:   # explicit inverse: n_c^2 doubles (else inside the tail)
        nc = H.level(nl - 1).A.num_rows
        assert cb["coarse"] >= 8 * nc * nc
    D.close()
