"""Per-rank compute floor of the row-partitioned N-GPU cycle, measured one rank at a time on one GPU.

    python tools/n8_floor.py [--n 400] [--ranks 8] [--agg 5000,20000,80000] [--reps 20] [--out f.json]

For each replicated-tail threshold (SSS_HIP_AGG_ROWS) and each rank r of an N-way partition of the
7-pt Poisson hierarchy, the rank's engine is built with the timing-only communicator
(sss_hip_comm_timing: every halo transfer, all-gather and all-reduce skipped; kernels, halo packs and
the graph exactly as over RCCL) and timed alone on the GPU:
  * cycle_ms: its captured V-cycle (graph replays), plus the local level-0 residual of the step;
  * per level: descent + ascent of an eager cycle (events between steps), and the replicated tail;
  * halo: exchanges per partitioned level per cycle and the doubles this rank sends in them.
The N-GPU step floor is the max over ranks of (cycle + residual); the exchange cost is modelled as
alpha per exchange (not overlapped) + bytes / beta, for a range of alpha, since RCCL point-to-point
latency between two MI355X cannot be measured on the one-GPU test box.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=400)
    p.add_argument("--stencil", type=int, default=7)
    p.add_argument("--ranks", type=int, default=8)
    p.add_argument("--agg", default="5000,20000,80000")
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--out", default="gpurun_out/n8_floor.json")
    p.add_argument("--single", type=int, default=1, help="also time the single-GPU engine's levels")
    p.add_argument("--only-ranks", default=None, help="comma list: time only these ranks")
    a = p.parse_args()
    import ctypes as C
    import amg_amd as A

    def log(m):
        print(f"[floor {time.strftime('%H:%M:%S')}] {m}", file=sys.stderr, flush=True)

    t0 = time.perf_counter()
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
    levels = [(H.level(l).A.num_rows, H.level(l).A.num_nnzs) for l in range(H.num_levels)]
    log(f"setup {time.perf_counter() - t0:.1f} s, levels {levels}")
    smoother = "hybrid" if a.stencil == 7 else "jacobi"
    one = None
    if a.single:   # the single-GPU engine's own per-level times on the same hierarchy
        S = A.DeviceHierarchy(H, smoother="hybrid" if a.stencil == 7 else "hybrid", coarse="direct", device=0)
        S.upload(0, "b", np.ones(levels[0][0]))
        S.upload(0, "x", np.ones(levels[0][0]))
        S.cycle()
        S.residual_norm()
        one = S.time_levels(a.reps)
        S.close()
        log(f"N = 1 per level (eager) {[round(x, 3) for x in one]}, sum {sum(one):.3f} ms")
    res = {"workload": f"poisson{a.stencil}_{a.n}^3", "ranks": a.ranks, "levels": levels, "reps": a.reps,
           "smoother": smoother, "single_gpu_level_ms": one, "by_agg": {}}
    for agg in [int(x) for x in a.agg.split(",")]:
        ranks = []
        for r in (range(a.ranks) if not a.only_ranks else [int(x) for x in a.only_ranks.split(",")]):
            comm = A.Comm(a.ranks, r, "timing", device=0)
            D = A.DistHierarchy(H, comm, smoother=smoother, coarse="direct", device=0, agg_rows=agg)
            own = D.hi - D.lo
            D.upload("b", np.ones(own))
            D.upload("x", np.ones(own))
            D.halo_stats(reset=True)
            D.cycle()                  # captures the graph: the halo counts of one cycle
            D.residual_norm()
            hs = D.halo_stats(reset=True)
            cyc, lv = D.time_levels(a.reps)
            res0 = D.time_level0_spmv(a.reps)
            tl = D.time_tail_levels(a.reps)[:hs["tail_levels"]]
            ranks.append({"rank": r, "rows": own, "nagg": D.nagg, "cycle_ms": cyc, "resid_ms": res0,
                          "level_ms": lv[:-1], "tail_ms": lv[-1], "tail_level_ms": tl, **hs})
            log(f"agg {agg} rank {r}: nagg {D.nagg}, cycle {cyc:.3f} ms (+ residual {res0:.3f}), tail {lv[-1]:.3f} ms, "
                f"exchanges {sum(hs['exchanges'])}")
            D.close()
            comm.close()
        nagg = ranks[0]["nagg"]
        floor = max(x["cycle_ms"] + x["resid_ms"] for x in ranks)
        per_level_max = [max(x["level_ms"][l] for x in ranks) for l in range(nagg)]
        tail = max(x["tail_ms"] for x in ranks)
        tail_levels_ms = [max(x["tail_level_ms"][k] for x in ranks) for k in range(len(ranks[0]["tail_level_ms"]))]
        ex = [max(x["exchanges"][l] for x in ranks) for l in range(nagg)]
        exb = [max(x["doubles_sent"][l] for x in ranks) * 8 for l in range(nagg)]
        n_ex = sum(ex) + 2   # + the tail all-gather and the norm all-reduce
        bytes_ex = sum(exb) + 8 * ranks[0]["gather_all"]
        model = {f"alpha_{int(al * 1e6)}us": floor + (n_ex * al + bytes_ex / 50e9) * 1e3 for al in (8e-6, 15e-6, 25e-6)}
        res["by_agg"][agg] = {"nagg": nagg, "tail_levels": ranks[0]["tail_levels"], "floor_ms": floor,
                              "per_level_max_ms": per_level_max, "tail_ms_max": tail, "tail_level_ms_max": tail_levels_ms,
                              "tail_share_of_eager_levels": tail / (sum(per_level_max) + tail),
                              "exchanges_per_cycle_max_rank": ex, "halo_bytes_per_cycle_max_rank": exb,
                              "gather_rows": ranks[0]["gather_all"], "exchanges_total": n_ex,
                              "predicted_step_ms": model, "ranks": ranks}
        log(f"agg {agg}: floor {floor:.3f} ms, {n_ex} exchanges, {bytes_ex / 1e6:.1f} MB; predicted {model}")
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))
    print(json.dumps({k: (v if k != "by_agg" else {g: {kk: vv for kk, vv in d.items() if kk != "ranks"}
                                                   for g, d in v.items()}) for k, v in res.items()}))


if __name__ == "__main__":
    main()
