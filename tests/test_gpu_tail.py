"""GPU: the V-cycle's small coarse levels as one single-workgroup launch (sss_tail.hip) give the
iterates of the per-level launches bit for bit (SSS_HIP_TAIL=1 vs 0), on hierarchies whose
coarsest levels qualify: the G3_circuit stand-in and 7-pt / 27-pt stencils in throughput mode."""
from __future__ import annotations

import numpy as np
import pytest

import amg_amd as A
from amg_amd import workloads as W
from conftest import build_hierarchy, quiet_ctx

pytestmark = pytest.mark.gpu


def _run(H, cycles, **kw):
    n = H.level(0).A.num_rows
    D = A.DeviceHierarchy(H, **kw)
    try:
        D.upload(0, "b", np.ones(n))
        D.upload(0, "x", np.ones(n))
        rel = []
        for _ in range(cycles):
            D.cycle()
            rel.append(D.residual_norm())
        return np.array(rel), D.download(0, "x")
    finally:
        D.close()


@pytest.mark.parametrize("case", ["circ60k", "p7_24", "a27_16"])
@pytest.mark.parametrize("graph", [1, 0])
def test_tail_bitwise(case, graph, monkeypatch):
    keep = None
    if case == "circ60k":
        keep = W.circuit_csr(60000)
        M = keep.mat
    elif case == "p7_24":
        M = A.generate(7, 24)
    else:
        M = A.generate(27, 16)
    H = build_hierarchy(M, quiet_ctx)
    monkeypatch.setenv("SSS_HIP_TAIL_NNZ", "1000000")   # every qualifying level, not only the tiny ones
    kw = dict(smoother="hybrid", coarse="direct", sum_order=1, graph=graph)
    out = {}
    for t in ("1", "0"):
        monkeypatch.setenv("SSS_HIP_TAIL", t)
        if t == "1":   # the tail does engage on these hierarchies
            D = A.DeviceHierarchy(H, **kw)
            assert A.lib().sss_hip_tail_from(D.h) > 0, case
            D.close()
        out[t] = _run(H, 6, **kw)
    assert np.array_equal(out["1"][0].view(np.uint64), out["0"][0].view(np.uint64))
    assert np.array_equal(out["1"][1].view(np.uint64), out["0"][1].view(np.uint64))
    del keep


def test_tail_engaged_on_circuit(monkeypatch):
    """The stand-in's coarsest levels do take the tail (its level table: 1,629 / 209 / 19 rows)."""
    keep = W.circuit_csr(W.G3_CIRCUIT_ROWS)
    H = build_hierarchy(keep.mat, quiet_ctx)
    monkeypatch.setenv("SSS_HIP_TAIL", "1")
    D = A.DeviceHierarchy(H, smoother="hybrid", coarse="direct", sum_order=1)
    try:
        assert A.lib().sss_hip_tail_from(D.h) > 0
    finally:
        D.close()
    del keep
