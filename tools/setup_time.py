"""Lab tool: time the host setup (SSS_amg_setup) of a 7-pt n^3 Poisson hierarchy; with
SSS_SETUP_TIMING=1 the per-level phases go to stderr.   python tools/setup_time.py --n 400"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=400)
    p.add_argument("--stencil", type=int, default=7)
    a = p.parse_args()
    import amg_amd as A
    M = A.generate(a.stencil, a.n)
    t0 = time.perf_counter()
    H = A.Hierarchy(M)
    print(f"[setup_time] n={a.n} setup {time.perf_counter() - t0:.2f} s, {H.num_levels} levels", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
