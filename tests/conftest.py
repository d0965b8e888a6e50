"""Shared test setup.

Markers:  gpu — needs a HIP device (run on the MI355X box: `pytest -m gpu`); everything else
runs on CPU here.  The product library and the oracle are built on first use if missing.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"
REF_MTX = Path("/root/reference/amg/Matrix/1138_bus.mtx")
BUS_MTX = GOLDEN / "1138_bus.mtx" if (GOLDEN / "1138_bus.mtx").exists() else REF_MTX


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) with the HIP runtime")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def _ensure_built():
    lib = ROOT / "amg_amd" / "lib" / "libsss_amg.so"
    ora = ROOT / "oracle" / "liboracle.so"
    if not lib.exists():
        subprocess.run(["make", "-j8"], cwd=ROOT, check=True, stdout=subprocess.DEVNULL)
    if not ora.exists():
        subprocess.run(["make", "oracle"], cwd=ROOT, check=True, stdout=subprocess.DEVNULL)


_ensure_built()

import amg_amd as A  # noqa: E402
import oracle  # noqa: E402
from amg_amd._native import dptr, iptr  # noqa: E402


def vec(a: np.ndarray) -> A.SSS_VEC:
    return A.SSS_VEC(len(a), dptr(a))


def seq_sum(a: np.ndarray) -> float:
    """Left-to-right sum (the reference's order), for 17-digit known-answer checks."""
    return float(np.cumsum(a)[-1]) if len(a) else 0.0


def oracle_solve(H, b: np.ndarray, x: np.ndarray, **kw):
    """Run the CPU oracle's SSS_amg_solve; returns (rtn, relres history)."""
    rel = np.zeros(128)
    ab = np.zeros(128)
    o = oracle.opts(**kw)
    rtn = oracle.load().ora_solve(C.byref(H.mg), C.byref(vec(x)), C.byref(vec(b)), C.byref(o), dptr(rel),
                                  dptr(ab), 128)
    return rtn, rel[: rtn.nits].copy(), ab[: rtn.nits].copy()


@pytest.fixture(scope="session")
def bus_matrix():
    return A.read_mtx(BUS_MTX)


class quiet_ctx:
    """Silence the C library's stdout chatter (setup prints) at the fd level."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        self.null = os.open(os.devnull, os.O_WRONLY)
        os.dup2(self.null, 1)

    def __exit__(self, *a):
        C.CDLL(None).fflush(None)
        os.dup2(self.saved, 1)
        os.close(self.saved)
        os.close(self.null)


@pytest.fixture(scope="session")
def quiet():
    return quiet_ctx


def build_hierarchy(M, quiet_cls):
    with quiet_cls():
        return A.Hierarchy(M)


def device_mode_oracle_opts(H, **device_kw) -> dict:
    """Oracle options (oracle.opts) of the per-level smoothers a DeviceHierarchy(H, **device_kw)
    actually runs -- throughput mode's hybrid keeps exact GS-CF on level 0 only when that level is
    chain-free, else the two-stage form there (sss_hier.hip hybrid0_two_stage).  Needs a GPU."""
    D = A.DeviceHierarchy(H, **device_kw)
    try:
        info = [D.level_info(l) for l in range(H.num_levels - 1)]
    finally:
        D.close()
    jac = [l for l, i in enumerate(info) if i.smoother_kind == 2]   # SSS_HIP_SMOOTH_JACOBI
    mask = sum(1 << l for l, i in enumerate(info) if i.inner > 0)
    steps = sorted({i.inner for i in info if i.inner > 0})
    assert len(steps) <= 2, steps   # the base count, and the long-row levels' (sss_hip_opts::inner_long)
    base = steps[0] if steps else 0
    kw = dict(smoother=1, jacobi_from=jac[0] if jac else len(info), inner=base,
              inner_mask=mask if mask else 1 << 30,
              inner_long=steps[-1] - base if steps else 0,
              long_mask=sum(1 << l for l, i in enumerate(info) if steps and i.inner == steps[-1] > base))
    if device_kw.get("coarse") == "direct":
        kw["coarse_mode"] = 1
    return kw
