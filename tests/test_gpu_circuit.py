"""Whole AMG solve on the irregular G3_circuit stand-in (amg_amd/workloads.py; BASELINE.json
configs[3]): the smoother, transfers and coarse solve on a ragged, heavy-tailed operator.

- parity mode (exact GS-CF, reference CG(beta=1)+GMRES coarse solve) at 50K rows: x bitwise the
  oracle's after every cycle, the relres history equal (level-0 norm reduced in tree order);
- throughput mode at the full 1,585,478 rows: converges below tol within the reference semantics'
  iteration count + 2 (SURVEY.md 8(c) ladder), that count measured by the parity engine on the
  same operator, and lands on the parity solution.
"""
from __future__ import annotations

import numpy as np
import pytest

import amg_amd as A
from amg_amd import workloads as W
from conftest import build_hierarchy, device_mode_oracle_opts, quiet_ctx
from test_gpu_parity import _gpu_history, _oracle_history

pytestmark = pytest.mark.gpu


def _hier(n):
    M = W.circuit_csr(n)   # owns the arrays M.mat points into: alive through the setup (which copies A)
    return build_hierarchy(M.mat, quiet_ctx)


@pytest.fixture(scope="module")
def circ50k():
    return _hier(50000)


@pytest.fixture(scope="module")
def circ_full():
    return _hier(W.G3_CIRCUIT_ROWS)


def test_circuit_parity_bitwise(circ50k):
    rel_r, x_r = _oracle_history(circ50k)
    rel_g, x_g = _gpu_history(circ50k)
    assert len(rel_g) == len(rel_r) and rel_r[-1] < circ50k.pars.tol
    assert np.array_equal(x_g.view(np.uint64), x_r.view(np.uint64))
    assert np.allclose(rel_g, rel_r, rtol=1e-13, atol=0)


def test_circuit_throughput_full_size(circ_full):
    H = circ_full
    rel_p, x_p = _gpu_history(H)   # reference semantics (bitwise the oracle's iterates)
    rel_t, x_t = _gpu_history(H, smoother="hybrid", coarse="direct")
    print(f"circuit 1.58M: parity {len(rel_p)} iterations (relres {rel_p[-1]:.3e}), throughput {len(rel_t)} "
          f"(relres {rel_t[-1]:.3e}), |x_t - x_p| / |x_p| = {np.linalg.norm(x_t - x_p) / np.linalg.norm(x_p):.3e}")
    assert rel_p[-1] < H.pars.tol and rel_t[-1] < H.pars.tol
    assert len(rel_t) <= len(rel_p) + 2
    assert np.linalg.norm(x_t - x_p) <= 1e-5 * np.linalg.norm(x_p)


@pytest.mark.parametrize("hname", ["p32", "a27", "circ"])
def test_hybrid_level0_rule(request, hname, circ50k):
    """Throughput mode's hybrid smoother keeps exact GS-CF on level 0 only where it is chain-free
    (7-pt: red-black classes); on a level 0 with same-class couplings (27-pt, the circuit operator)
    that level runs the two-stage form instead.  The device's choice is reported per level and its
    iterates follow the oracle in the same per-level configuration."""
    H = {"p32": lambda: _hier_stencil(7, 32), "a27": lambda: _hier_stencil(27, 16), "circ": lambda: circ50k}[hname]()
    D = A.DeviceHierarchy(H, smoother="hybrid", coarse="direct")
    try:
        info = [D.level_info(l) for l in range(H.num_levels - 1)]
    finally:
        D.close()
    k0, i0 = info[0].smoother_kind, info[0].inner
    if hname == "p32":
        assert (k0, i0) == (0, 0)
    else:
        assert k0 == 2 and i0 >= 1
    assert all(i.smoother_kind == 2 for i in info[1:])
    kw = device_mode_oracle_opts(H, smoother="hybrid", coarse="direct")
    assert kw["jacobi_from"] == (1 if hname == "p32" else 0)
    rel_o, x_o = _oracle_history(H, **kw)
    rel_g, x_g = _gpu_history(H, smoother="hybrid", coarse="direct")
    assert len(rel_g) == len(rel_o) and rel_g[-1] < H.pars.tol
    assert np.allclose(rel_g, rel_o, rtol=1e-6)
    rel_ref, _ = _oracle_history(H)
    assert len(rel_g) <= len(rel_ref) + 2


def _hier_stencil(kind, n):
    return build_hierarchy(A.generate(kind, n), quiet_ctx)
