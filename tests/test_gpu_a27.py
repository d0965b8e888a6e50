"""The 27-point anisotropic operator (BASELINE.json configs[4]; SURVEY.md 8(d): -1 in-plane,
-0.1 across planes, diagonal 9.8) at 64^3 on the GPU.

Its level 0 is not red-black (same-class couplings), so the exact GS-CF passes there have chains:
  * parity mode (exact GS-CF on every level, the reference's CG(beta=1)+GMRES coarse solve): x is
    bitwise the oracle's whole solve (ora_solve, Solve/SSS_SOLVE.c:4-87 restated) after the same
    number of iterations, the relres history within 1e-13;
  * throughput mode, hybrid (two-stage GS-CF on level 0 since its classes are coupled): converges
    within the reference's count + 2;
  * the 4-rank configuration's smoother (bench.py N = 4: C/F-Jacobi on level 0, whose GS-CF
    chains would cross ranks): also within the reference's count + 2, on one GPU and row-partitioned
    over 4 ranks (tests/test_dist_gpu.py covers the partitioned iterates bitwise).
"""
from __future__ import annotations

import numpy as np
import pytest

import amg_amd as A
from conftest import build_hierarchy, oracle_solve

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def a64_h(quiet):
    return build_hierarchy(A.generate(27, 64), quiet)


@pytest.fixture(scope="module")
def ref64(a64_h):
    n = a64_h.level(0).A.num_rows
    x = np.ones(n)
    rtn, rel, _ = oracle_solve(a64_h, np.ones(n), x)
    return rtn, rel, x


def _solve(H, max_it, stop=True, **kw):
    n = H.level(0).A.num_rows
    D = A.DeviceHierarchy(H, device=0, **kw)
    try:
        D.upload(0, "b", np.ones(n))
        D.upload(0, "x", np.ones(n))
        rel = []
        for _ in range(max_it):
            D.cycle()
            rel.append(D.residual_norm() / np.sqrt(n))
            if stop and rel[-1] < H.pars.tol:
                break
        return rel, D.download(0, "x")
    finally:
        D.close()


def test_levels_have_chains(a64_h):
    """Level 0 of the 27-point operator couples points of one class (not red-black)."""
    rp, ci, _ = A.csr_arrays(a64_h.level(0).A)
    mark = np.ctypeslib.as_array(a64_h.level(0).cfmark.d, shape=(a64_h.level(0).A.num_rows,))
    rows = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
    same = (mark[rows] == 1) == (mark[ci] == 1)
    assert np.any(same & (rows != ci))


@pytest.mark.timeout(600)
def test_parity_solve_bitwise_a27_64(a64_h, ref64):
    rtn, rel_r, x_r = ref64
    rel, x = _solve(a64_h, len(rel_r), stop=False, smoother="exact", coarse="krylov", sum_order=0)
    assert np.array_equal(x.view(np.uint64), x_r.view(np.uint64))
    assert np.allclose(rel, rel_r, rtol=1e-13, atol=0)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("smoother", ["hybrid", "jacobi"])
def test_throughput_ladder_a27_64(a64_h, ref64, smoother):
    rtn, rel_r, x_r = ref64
    rel, x = _solve(a64_h, 40, smoother=smoother, coarse="direct", sum_order=1)
    assert rel[-1] < a64_h.pars.tol
    assert len(rel) <= len(rel_r) + 2, (smoother, len(rel), len(rel_r))
    assert np.linalg.norm(x - x_r) <= 1e-5 * np.linalg.norm(x_r)
