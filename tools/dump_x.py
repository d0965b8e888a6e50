"""x after K V-cycles of the throughput engine on a stencil problem, saved for a bitwise A/B of two
builds of the library (SSS_AMG_LIB selects the one loaded).

    python tools/dump_x.py --n 256 --stencil 7 --cycles 4 --out x.npy
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=256)
    p.add_argument("--stencil", type=int, default=7)
    p.add_argument("--cycles", type=int, default=4)
    p.add_argument("--smoother", default="hybrid")
    p.add_argument("--out", required=True)
    a = p.parse_args()
    import amg_amd as A
    M = A.generate(a.stencil, a.n)
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        H = A.Hierarchy(M)
    finally:
        C.CDLL(None).fflush(None)
        os.dup2(saved, 1)
        os.close(saved)
    A.lib().SSS_mat_destroy(C.byref(M))
    n = H.level(0).A.num_rows
    D = A.DeviceHierarchy(H, smoother=a.smoother, coarse="direct")
    D.upload(0, "b", np.ones(n))
    D.upload(0, "x", np.ones(n))
    rel = []
    for _ in range(a.cycles):
        D.cycle()
        rel.append(D.residual_norm())
    np.save(a.out, D.download(0, "x"))
    print(a.out, rel, flush=True)


if __name__ == "__main__":
    main()
