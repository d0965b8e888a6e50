"""Per-(kernel, grid) summary of a rocprofv3 kernel trace (rocpd .db).

    python tools/launch_shapes.py gpurun_out/prof_cur/run_results.db [out.txt]

One kernel template serves every level (and, for the residual, the full level-0 SpMV and its F-row
half), so rocprofv3's per-name `--stats` average mixes launch sizes.  Grouping by the grid size
separates them: the level-0 residual SpMV that bench.py times is `spmv_adaptive<2, false>` with
one workgroup per row block of A0 (250,000 at 400^3).
"""
from __future__ import annotations

import sqlite3
import sys
from collections import defaultdict


def main():
    c = sqlite3.connect(sys.argv[1])
    agg = defaultdict(lambda: [0, 0.0])
    for name, gx, wx, dur in c.execute("select name, grid_x, workgroup_x, end - start from kernels"):
        k = (name.split("(")[0], gx // max(wx, 1))
        agg[k][0] += 1
        agg[k][1] += dur / 1e3
    lines = ["# kernel, workgroups, calls, avg_us, total_ms   (sorted by total)"]
    for (nm, wg), (cnt, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"{nm:45s} workgroups={wg:9d} calls={cnt:6d} avg_us={tot / cnt:10.1f} total_ms={tot / 1e3:9.2f}")
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(text)
    else:
        sys.stdout.write(text)


if __name__ == "__main__":
    main()
