"""Setup with the HBM mirror built while it runs (sss_hip_setup_create).

The pipelined entry must give exactly what SSS_amg_setup followed by sss_hip_hier_create gives:
the same host hierarchy (every level's A, P, R and C/F marks, bit for bit) and a mirror whose
iterates are bitwise those of the sequentially built one, in both engine modes, on a stencil
operator, a 27-point operator and the irregular circuit stand-in (whose relabeling, two-stage and
free-order uploads differ per level).
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import amg_amd as A
from amg_amd import workloads as W
from conftest import BUS_MTX, build_hierarchy, quiet_ctx

pytestmark = pytest.mark.gpu


def _digest(H) -> str:
    h = hashlib.sha256()
    for l in range(H.num_levels):
        L = H.level(l)
        n, nnz = L.A.num_rows, L.A.num_nnzs
        h.update(np.ctypeslib.as_array(L.A.row_ptr, shape=(n + 1,)).tobytes())
        h.update(np.ctypeslib.as_array(L.A.col_idx, shape=(nnz,)).tobytes())
        h.update(np.ctypeslib.as_array(L.A.val, shape=(nnz,)).tobytes())
        if l + 1 < H.num_levels:
            h.update(np.ctypeslib.as_array(L.cfmark.d, shape=(n,)).tobytes())
            for M in (L.P, L.R):
                h.update(np.ctypeslib.as_array(M.row_ptr, shape=(M.num_rows + 1,)).tobytes())
                h.update(np.ctypeslib.as_array(M.val, shape=(M.num_nnzs,)).tobytes())
    return h.hexdigest()


def _iterate(D, n, cycles=4):
    D.upload(0, "b", np.ones(n))
    D.upload(0, "x", np.ones(n))
    rel = []
    for _ in range(cycles):
        D.cycle()
        rel.append(D.residual_norm())
    return np.array(rel), D.download(0, "x")


@pytest.mark.parametrize("case", ["p7_40", "a27_16", "circ60k", "bus"])
@pytest.mark.parametrize("mode", [("exact", "krylov"), ("hybrid", "direct")])
def test_pipelined_setup_matches_sequential(case, mode):
    keep = None
    if case == "bus":
        M = A.read_mtx(BUS_MTX)
    elif case.startswith("p7"):
        M = A.generate(7, 40)
    elif case.startswith("a27"):
        M = A.generate(27, 16)
    else:
        keep = W.circuit_csr(60000)
        M = keep.mat
    smoother, coarse = mode
    H_seq = build_hierarchy(M, quiet_ctx)
    n = H_seq.level(0).A.num_rows
    D_seq = A.DeviceHierarchy(H_seq, smoother=smoother, coarse=coarse)
    rel_s, x_s = _iterate(D_seq, n)
    D_seq.close()
    with quiet_ctx():
        D_pip = A.DeviceHierarchy(None, smoother=smoother, coarse=coarse, setup_from=M)
    H_pip = D_pip.H
    assert H_pip.num_levels == H_seq.num_levels
    assert _digest(H_pip) == _digest(H_seq)
    assert len(D_pip.times) == 3 and D_pip.times[0] > 0
    rel_p, x_p = _iterate(D_pip, n)
    D_pip.close()
    assert np.array_equal(rel_p.view(np.uint64), rel_s.view(np.uint64))
    assert np.array_equal(x_p.view(np.uint64), x_s.view(np.uint64))
    del keep


@pytest.mark.parametrize("case", ["p7_32", "a27_16", "circ60k"])
@pytest.mark.parametrize("merge_g", ["4", "8"])
def test_device_builders_match_host(case, merge_g, monkeypatch):
    """The free-order formats built on the GPU (sss_build.hip: merged row groups and column-sorted
    rows by a segmented radix sort of the resident CSR) are the host builders' bit for bit: with
    every level on the free-order kernels (SSS_HIP_FREE_MIN=1) and merged groups wherever possible,
    the throughput-mode iterates (tree-order sums over those formats) are identical either way."""
    keep = None
    if case.startswith("p7"):
        M = A.generate(7, 32)
    elif case.startswith("a27"):
        M = A.generate(27, 16)
    else:
        keep = W.circuit_csr(60000)
        M = keep.mat
    H = build_hierarchy(M, quiet_ctx)
    n = H.level(0).A.num_rows
    monkeypatch.setenv("SSS_HIP_FREE_MIN", "1")
    monkeypatch.setenv("SSS_HIP_MERGE_MIN_ROWS", "1")
    monkeypatch.setenv("SSS_HIP_MERGE_G", merge_g)
    out = {}
    for build in ("1", "0"):
        monkeypatch.setenv("SSS_HIP_GPU_BUILD", build)
        D = A.DeviceHierarchy(H, smoother="hybrid", coarse="direct", sum_order=1)
        assert any(D.level_info(l).a_format & 8 for l in range(H.num_levels - 1))   # merged copies exist
        out[build] = _iterate(D, n, cycles=6)
        D.close()
    assert np.array_equal(out["1"][0].view(np.uint64), out["0"][0].view(np.uint64))
    assert np.array_equal(out["1"][1].view(np.uint64), out["0"][1].view(np.uint64))
    del keep
