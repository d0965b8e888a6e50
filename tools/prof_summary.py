"""Summarise a rocprofv3 kernel trace (rocpd SQLite .db or kernel_trace.csv).

    python tools/prof_summary.py gpurun_out/prof_r1/run_results.db [--stats out.csv] [--shapes out.txt]

--stats  per-kernel totals (Name, Calls, TotalDurationNs, AverageNs, MinNs, MaxNs, Percentage), the
         layout of rocprofv3 --stats' kernel_stats.csv
--shapes per (kernel, workgroups) group, which separates the levels of the hierarchy
"""
from __future__ import annotations

import argparse
import csv
import sqlite3
from collections import defaultdict


def load(path: str):
    rows = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, dur, gx, wx in c.execute("select name, duration, grid_x, workgroup_x from kernels"):
            rows.append((name, int(dur), int(gx) // max(int(wx), 1)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                rows.append((r["Kernel_Name"], dur, int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--stats")
    ap.add_argument("--shapes")
    ap.add_argument("--header", default="")
    a = ap.parse_args()
    rows = load(a.trace)
    total = sum(d for _, d, _ in rows) or 1
    per = defaultdict(list)
    shape = defaultdict(list)
    for n, d, g in rows:
        per[n].append(d)
        shape[(n, g)].append(d)
    out = [("Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage")]
    for n, ds in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        out.append((n, len(ds), sum(ds), sum(ds) / len(ds), min(ds), max(ds), 100.0 * sum(ds) / total))
    if a.stats:
        with open(a.stats, "w", newline="") as f:
            csv.writer(f).writerows(out)
    lines = [a.header] if a.header else []
    for (n, g), ds in sorted(shape.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"{n[:44]:44s}  workgroups={g:9d} calls={len(ds):5d} avg_us={sum(ds)/len(ds)/1e3:10.1f} "
                     f"total_ms={sum(ds)/1e6:9.2f}")
    txt = "\n".join(lines) + "\n"
    if a.shapes:
        with open(a.shapes, "w") as f:
            f.write(txt)
    else:
        print(txt)


if __name__ == "__main__":
    main()
