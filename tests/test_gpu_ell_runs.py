"""GPU: run-coded dictionary ELL blocks (DevCSR::dv_rs / dv_rc) are bitwise-neutral.

A W = 8 dictionary ELL block whose rows form at most kEllRuns runs of equal code bytes stores each
run's codes once; its rows read them from LDS instead of one 8-byte load per row.  The codes are the
same bytes, so every product, chain and epilogue is unchanged: with SSS_HIP_ELL_RUNS=0/1 the iterates,
the in-cycle residual and the outer norms must be bitwise equal.  7-pt 96^3 (48 F rows per grid line:
every level-0 block fits) and 64^3 (32 per line: some blocks fit, some keep per-row codes -- the
mixed path, including the two-rows-per-thread relaxation with one run-coded block of its pair)."""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import amg_amd as A  # noqa: E402
from conftest import build_hierarchy, quiet_ctx  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[(96, ""), (96, "11"), (64, "")])
def grid_h(request):
    edge, cap = request.param
    H = build_hierarchy(A.generate(7, edge), quiet_ctx)
    yield edge, cap, H
    H.close()


@pytest.mark.parametrize("smoother,coarse,cycles", [("hybrid", "direct", 4), ("exact", "direct", 2)])
def test_ell_runs_bitwise(grid_h, smoother, coarse, cycles, monkeypatch):
    edge, cap, H = grid_h
    n = H.level(0).A.num_rows
    out = []
    for on in (cap, "0"):
        monkeypatch.setenv("SSS_HIP_ELL_RUNS", on)
        D = A.DeviceHierarchy(H, smoother=smoother, coarse=coarse, device=0)
        info = D.level_info(0)
        if on != "0":
            assert info.a_format & 64, "level 0 is not a dictionary ELL"
            assert 0 < info.a_run_rows <= n, info.a_run_rows
            if cap:
                assert info.a_run_rows < n    # the mixed path
            else:
                assert info.a_run_rows == n   # every block fits kEllRuns runs
        else:
            assert info.a_run_rows == 0
        D.upload(0, "b", np.ones(n))
        D.upload(0, "x", np.ones(n))
        norms = []
        for _ in range(cycles):
            D.cycle()
            norms.append(D.residual_norm())
        out.append((np.array(norms), D.download(0, "x"), D.download(0, "wp"), info.r_run_rows))
        D.close()
    (n1, x1, w1, rr1), (n0, x0, w0, _) = out
    assert np.array_equal(n1.view(np.uint64), n0.view(np.uint64))
    assert np.array_equal(x1.view(np.uint64), x0.view(np.uint64))
    assert np.array_equal(w1.view(np.uint64), w0.view(np.uint64))
