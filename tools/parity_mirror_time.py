"""Lab tool (GPU box): phases of building the parity-mode HBM mirror (exact GS-CF everywhere, device
Krylov coarse solve) of a 7-pt Poisson hierarchy -- SSS_HIP_TIMING=2 prints each level's relabel,
uploads and smoother-plan phases on stderr.

    SSS_HIP_TIMING=2 python tools/parity_mirror_time.py --n 400
"""
from __future__ import annotations

import argparse
import ctypes as C
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=400)
    a = p.parse_args()
    import amg_amd as A
    t0 = time.perf_counter()
    M = A.generate(7, a.n)
    H = A.Hierarchy(M)
    A.lib().SSS_mat_destroy(C.byref(M))
    print(f"[pm] setup {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    t1 = time.perf_counter()
    D = A.DeviceHierarchy(H, smoother="exact", coarse="krylov", device=0, sum_order=0)
    print(f"[pm] parity mirror {time.perf_counter() - t1:.1f} s", file=sys.stderr, flush=True)
    D.close()


if __name__ == "__main__":
    main()
