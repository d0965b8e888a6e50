"""Lab tool (GPU box): time the exact GS-CF pre-smoother (2 sweeps) of every level per engine.

    python tools/gs_level_times.py --n 256 --engines launch,flow,fused,cu [--reps 3]

Prints one line per (engine, level): rows, F/C depth, chosen engines, ms per smoother call.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=256)
    p.add_argument("--stencil", type=int, default=7)
    p.add_argument("--engines", default="launch,flow,cu")
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--levels", default="")
    p.add_argument("--json", default=None)
    p.add_argument("--workload", default="stencil", choices=["stencil", "circuit"])
    p.add_argument("--rows", type=int, default=0, help="circuit stand-in rows (default: G3_circuit's)")
    a = p.parse_args()
    import amg_amd as A
    t0 = time.perf_counter()
    if a.workload == "circuit":
        from amg_amd import workloads as W
        keep = W.circuit_csr(a.rows or W.G3_CIRCUIT_ROWS)
        H = A.Hierarchy(keep.mat)
    else:
        M = A.generate(a.stencil, a.n)
        H = A.Hierarchy(M)
        A.lib().SSS_mat_destroy(C.byref(M))
    print(f"[gs] setup {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    levels = [int(x) for x in a.levels.split(",")] if a.levels else list(range(1, H.num_levels - 1))
    out = []
    for eng in a.engines.split(","):
        lab = ""
        if "+" in eng:   # lab: engine+VAR=VALUE[+VAR=VALUE...] sets environment variables for that run
            eng, lab = eng.split("+", 1)
            for kv in lab.split("+"):
                k, v = kv.split("=", 1)
                os.environ[k] = v
        os.environ["SSS_HIP_GS_ENGINE"] = "flow" if eng == "fused" else eng   # fused: all passes in one launch
        os.environ["SSS_HIP_GS_FUSED"] = "1" if eng == "fused" else "0"
        D = A.DeviceHierarchy(H, smoother="exact", coarse="direct", device=0)
        rng = np.random.default_rng(1)
        for l in levels:
            n = H.level(l).A.num_rows
            D.upload(l, "b", rng.standard_normal(n))
            D.upload(l, "x", rng.standard_normal(n))
            D.smooth(l, False)
            D.sync()
            ts = []
            for _ in range(a.reps):
                t1 = time.perf_counter()
                D.smooth(l, False)
                D.sync()
                ts.append(time.perf_counter() - t1)
            info = D.level_info(l)
            rec = {"engine": eng + ("+" + lab if lab else ""), "level": l, "rows": n, "nnz": H.level(l).A.num_nnzs, "dag_f": info.dag_f,
                   "dag_c": info.dag_c, "eng_f": info.gs_engine_f, "eng_c": info.gs_engine_c,
                   "stall": info.gs_stall, "ms": float(np.median(ts) * 1e3)}
            out.append(rec)
            print(f"[gs] {rec['engine']:6s} L{l} rows {n:9d} nnz/row {rec['nnz'] / n:7.1f} depth F/C {info.dag_f:5d}/{info.dag_c:5d} "
                  f"eng {info.gs_engine_f}/{info.gs_engine_c} stall {info.gs_stall}  {rec['ms']:9.2f} ms", file=sys.stderr,
                  flush=True)
        D.close()
        for kv in lab.split("+") if lab else []:
            os.environ.pop(kv.split("=", 1)[0], None)
    if a.json:
        Path(a.json).write_text(json.dumps(out))


if __name__ == "__main__":
    main()
