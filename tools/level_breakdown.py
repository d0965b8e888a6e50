"""Per-level time of one V-cycle from a rocprofv3 kernel trace (rocpd .db).

    python tools/level_breakdown.py gpurun_out/prof_x/run_results.db [bench.json]

Walks the kernels in start order.  A cycle ends at the residual-norm kernel
(spmv_*<2, true>, or relax_range<3> when it also computes the next first F pass); inside a cycle, a restriction (spmv_*<0, ...>, SSS_HIP_SPMV_MXY) moves the
level counter down, a prolongation (spmv_*<1, ...> or prolong_inject) moves it up, the dense GEMV / Krylov kernels
are the coarsest level.  Prints, per level, the kernel time of one average cycle split into
smoother / residual / restriction / prolongation / other, and, when the bench JSON (its
`config.hierarchy`) is given, the effective GB/s of 5 passes over the level's matrix
(4 smoother sweeps + 1 residual at 12 B per nonzero; vectors and transfers not counted).
"""
from __future__ import annotations

import json
import re
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    hier = None
    if len(sys.argv) > 2:
        with open(sys.argv[2]) as f:
            for line in f:
                if line.startswith("{"):
                    hier = json.loads(line)["config"]["hierarchy"]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    # drop everything before the first cycle: upload / explicit inverse; start after the first residual norm
    cycles = []
    cur = None
    lvl = 0
    for name, s, e in rows:
        dur = (e - s) / 1e3   # us
        m = re.search(r"(spmv_\w+)<(\d), (true|false)(?:, \w+)?>", name)
        # the outer residual norm ends a cycle: the fused-norm SpMV, or relax_range<3> (its F half
        # fused with the next cycle's first F pass, SmootherPlan::pend_ok)
        if (m and m.group(2) == "2" and m.group(3) == "true") or "relax_range<3" in name:
            if cur is not None:
                cur[("out", "resid")] += dur
                cycles.append(cur)
            cur = defaultdict(float)
            lvl = 0
            continue
        if cur is None:
            continue
        if "gj_" in name:
            continue
        if m:
            op = int(m.group(2))
            if op == 0:
                cur[(lvl, "restrict")] += dur
                lvl += 1
            elif op == 1:
                lvl -= 1
                cur[(lvl, "prolong")] += dur
            else:
                cur[(lvl, "resid")] += dur
            continue
        if "prolong_inject" in name:   # the C-row prolongation of a P whose C rows are injections
            lvl -= 1
            cur[(lvl, "prolong")] += dur
            continue
        if "dense_gemv" in name or "k_" in name.split("(")[0]:
            cur[("coarse", "solve")] += dur
            continue
        if any(k in name for k in ("relax", "ts_", "gs_", "scatter", "zero_first_pass")):
            cur[(lvl, "smooth")] += dur
        else:
            cur[(lvl, "other")] += dur
    # the last partial cycle (timed SpMV repetitions) is discarded; only complete cycles count
    cycles = [cy for cy in cycles if any(k[1] == "smooth" for k in cy)]
    nc = len(cycles)
    if not nc:
        print("no complete cycles found")
        return
    tot = defaultdict(float)
    for cy in cycles:
        for k, v in cy.items():
            tot[k] += v / nc
    levels = sorted({k[0] for k in tot if isinstance(k[0], int)})
    kinds = ["smooth", "resid", "restrict", "prolong", "other"]
    print(f"{nc} cycles; average kernel microseconds per cycle")
    print("level " + "".join(f"{k:>10}" for k in kinds) + f"{'total':>10}" + ("   5xA GB/s" if hier else ""))
    grand = 0.0
    for l in levels:
        vals = [tot.get((l, k), 0.0) for k in kinds]
        t = sum(vals)
        grand += t
        extra = ""
        if hier and l < len(hier):
            nnz = hier[l][1]
            extra = f"   {5 * 12 * nnz / (t * 1e-6) / 1e9:9.0f}"
        print(f"{l:5d} " + "".join(f"{v:10.1f}" for v in vals) + f"{t:10.1f}" + extra)
    for k in (("coarse", "solve"), ("out", "resid")):
        grand += tot.get(k, 0.0)
        print(f"{k[0]:>6} {tot.get(k, 0.0):10.1f}")
    print(f"total {grand:10.1f} us")


if __name__ == "__main__":
    main()
