"""Convergence study: outer-iteration relres histories and per-iteration times of several engine
modes on one 7-pt Poisson hierarchy (GPU box).  Lab tool, not product.

    python tools/conv_study.py --n 256 --modes parity,exact-direct,throughput [--json out.json]

Each mode: smoother[/coarse][/inner/inner_from][/sum_order], e.g.
  parity        exact GS-CF + reference CG(beta=1)+GMRES   (x bitwise the reference's)
  exact-direct  exact GS-CF + explicit-inverse coarse solve
  throughput    bench default (hybrid, direct, inner 1 from level 2, tree long-row sums)
  hyb:I:F[:L]   hybrid with I inner steps from level F, L more on long-row levels (default 1;
                direct coarse, tree sums)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def mode_kwargs(m: str) -> dict:
    if m == "parity":
        return dict(smoother="exact", coarse="krylov", sum_order=0)
    if m == "exact-direct":
        return dict(smoother="exact", coarse="direct", sum_order=0)
    if m == "throughput":
        return dict(smoother="hybrid", coarse="direct", sum_order=1)
    if m.startswith("hyb:"):   # hyb:I:F[:L] -- L extra inner steps on the long-row levels (default 1)
        f = m.split(":")
        return dict(smoother="hybrid", coarse="direct", sum_order=1, inner=int(f[1]), inner_from=int(f[2]),
                    inner_long=int(f[3]) if len(f) > 3 else 1)
    if m.startswith("mc"):
        return dict(smoother="multicolor", coarse="direct", sum_order=1)
    raise ValueError(m)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=256)
    p.add_argument("--stencil", type=int, default=7)
    p.add_argument("--modes", default="parity,throughput")
    p.add_argument("--maxit", type=int, default=40)
    p.add_argument("--json", default=None)
    a = p.parse_args()
    import amg_amd as A
    t0 = time.perf_counter()
    M = A.generate(a.stencil, a.n)
    H = A.Hierarchy(M)
    A.lib().SSS_mat_destroy(C.byref(M))
    N = H.level(0).A.num_rows
    print(f"[conv] setup {time.perf_counter() - t0:.1f} s, {H.num_levels} levels", file=sys.stderr, flush=True)
    out = {"n": a.n, "stencil": a.stencil, "levels": [(H.level(l).A.num_rows, H.level(l).A.num_nnzs)
                                                      for l in range(H.num_levels)], "modes": {}}
    normb = float(np.sqrt(N))
    import os
    for m in a.modes.split(","):
        base, _, eng = m.partition("@")   # parity@cu: exact GS engine override (SSS_HIP_GS_ENGINE)
        if eng:
            os.environ["SSS_HIP_GS_ENGINE"] = eng
        else:
            os.environ.pop("SSS_HIP_GS_ENGINE", None)
        t0 = time.perf_counter()
        D = A.DeviceHierarchy(H, device=0, **mode_kwargs(base))
        up = time.perf_counter() - t0
        D.upload(0, "b", np.ones(N))
        D.upload(0, "x", np.ones(N))
        hist, times = [], []
        for it in range(a.maxit):
            t1 = time.perf_counter()
            D.cycle()
            rel = D.residual_norm() / normb
            times.append(time.perf_counter() - t1)
            hist.append(rel)
            print(f"[conv] {m} it {it + 1}: relres {rel:.6e}  {times[-1] * 1e3:.2f} ms", file=sys.stderr, flush=True)
            if rel < H.pars.tol or not np.isfinite(rel):
                break
        x = D.download(0, "x")
        info = [D.level_info(l) for l in range(H.num_levels - 1)]
        engines = [(i.gs_engine_f, i.gs_engine_c) for i in info]
        stall = any(i.gs_stall for i in info)
        D.close()
        out["modes"][m] = {"upload_s": up, "relres": hist, "iters": len(hist),
                           "ms_per_iter_median": float(np.median(times) * 1e3), "gs_engines": engines,
                           "gs_stall": stall,
                           "sum_x": float(x.sum()), "x_sample": x[:: max(1, N // 4096)].tolist()}
        print(f"[conv] {m}: {len(hist)} iterations, upload {up:.1f} s, median {np.median(times) * 1e3:.2f} ms, "
              f"gs engines {engines}, stall {stall}", file=sys.stderr, flush=True)
    # pairwise x differences (sampled) against the first mode
    modes = list(out["modes"])
    if modes:
        ref = np.array(out["modes"][modes[0]]["x_sample"])
        for m in modes[1:]:
            xs = np.array(out["modes"][m]["x_sample"])
            out["modes"][m]["xdiff_vs_" + modes[0]] = float(np.linalg.norm(xs - ref) / np.linalg.norm(ref))
    for m in modes:
        out["modes"][m].pop("x_sample")
    s = json.dumps(out)
    print(s, flush=True)
    if a.json:
        Path(a.json).write_text(s)


if __name__ == "__main__":
    main()
