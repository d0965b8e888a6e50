"""Per-level time of one V-cycle from a rocprofv3 kernel trace (rocpd .db).

    python tools/level_breakdown.py gpurun_out/prof_x/run_results.db [bench.json]

Walks the kernels in start order.  A cycle ends at the residual-norm kernel
(spmv_*<2, true>, or relax_range<3> when it also computes the next first F pass); inside a cycle, a restriction (spmv_*<0, ...>, SSS_HIP_SPMV_MXY) moves the
level counter down, a prolongation (spmv_*<1, ...> or prolong_inject) moves it up, the dense GEMV / Krylov kernels
are the coarsest level.  Prints, per level, the kernel time of one average cycle split into
smoother / residual / restriction / prolongation / other, and, when the bench JSON is given, each
level's stored-format rate: the bytes its launches read and write in the engine's stored formats
(`vcycle_stored.bytes_per_level`, sss_hip_cycle_bytes) over its kernel time, and the same for the
outer residual, the coarsest solve and the whole cycle (kernel time, not the step's wall time).
"""
from __future__ import annotations

import json
import re
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    stored = None
    if len(sys.argv) > 2:
        with open(sys.argv[2]) as f:
            for line in f:
                if line.startswith("{"):
                    stored = json.loads(line).get("vcycle_stored")
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
    print("level " + "".join(f"{k:>10}" for k in kinds) + f"{'total':>10}" +
          ("   stored GB   GB/s  frac" if stored else ""))
    per = stored["bytes_per_level"] if stored else []

    def rate(nbytes, t):
        if not stored or t <= 0:
            return ""
        g = nbytes / (t * 1e-6) / 1e9
        return f"   {nbytes / 1e9:9.3f} {g:6.0f} {g / 8000.0:5.2f}"

    grand = 0.0
    for l in levels:
        vals = [tot.get((l, k), 0.0) for k in kinds]
        t = sum(vals)
        grand += t
        print(f"{l:5d} " + "".join(f"{v:10.1f}" for v in vals) + f"{t:10.1f}" + (rate(per[l], t) if l < len(per) else ""))
    for k, key in ((("coarse", "solve"), "bytes_coarse"), (("out", "resid"), "bytes_outer_residual")):
        t = tot.get(k, 0.0)
        grand += t
        print(f"{k[0]:>6} {t:10.1f}" + (" " * 50 + rate(stored[key], t) if stored else ""))
    print(f"total {grand:10.1f} us" + (" " * 44 + rate(stored["bytes_per_step"], grand) if stored else ""))


if __name__ == "__main__":
    main()
