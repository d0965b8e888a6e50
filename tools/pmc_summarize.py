"""Level-0 SpMV HBM traffic from the two rocprofv3 --pmc passes of tools/gpu/pmc.sh.

    python tools/pmc_summarize.py gpurun_out profiles/r02_level0_spmv_pmc.json

Reads gpurun_out/pmc_FETCH_SIZE/**.csv and gpurun_out/pmc_WRITE_SIZE/**.csv (one row per launch),
keeps the level-0 residual SpMV launches (spmv_adaptive<2, ...>, the kernel tools/pmc_level0.py
times), and writes the per-launch HBM bytes with the gfx950 FETCH_SIZE correction of
MI355X_MICROARCH.md (coalesced streaming reads report half their bytes; re-measured with
tools/pmc_calib.hip, profiles/r01_pmc/calibration_fetch_size.csv).  The format and algorithmic
bytes come from the JSON line pmc_level0.py printed into gpurun_out/pmc_FETCH_SIZE.log.
"""
from __future__ import annotations

import csv
import json
import sys
from pathlib import Path

FETCH_CORRECTION = 2.0


def counter_avg(d: Path, name: str) -> tuple[float, int]:
    vals = []
    for f in d.rglob("*.csv"):
        with open(f) as fh:
            rd = csv.DictReader(fh)
            if "Counter_Name" not in (rd.fieldnames or []):
                continue
            for r in rd:
                if r["Counter_Name"] == name and "spmv_adaptive<2" in r["Kernel_Name"]:
                    vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {name} rows for spmv_adaptive<2, ...> under {d}")
    return sum(vals) / len(vals), len(vals)


def main():
    out = Path(sys.argv[1])
    dst = Path(sys.argv[2])
    info = None
    for line in (out / "pmc_FETCH_SIZE.log").read_text().splitlines():
        if line.startswith("{"):
            info = json.loads(line)
    if info is None:
        raise SystemExit("pmc_level0.py JSON line not found")
    fetch, nf = counter_avg(out / "pmc_FETCH_SIZE", "FETCH_SIZE")
    write, nw = counter_avg(out / "pmc_WRITE_SIZE", "WRITE_SIZE")
    rd = fetch * 1024 * FETCH_CORRECTION
    wr = write * 1024
    alg = info["algorithmic_bytes_per_launch"]
    rec = {
        "n": info["n"], "rows": info["rows"], "nnz": info["nnz"], "a_format": info["a_format"],
        "kernel": "spmv_adaptive<RESID> level 0 (bench roofline kernel)",
        "avg_ms_unprofiled": info["avg_ms"],
        "fetch_size_kib_raw": fetch, "write_size_kib_raw": write, "fetch_correction": FETCH_CORRECTION,
        "correction_source": "MI355X_MICROARCH.md HBM section; re-measured with tools/pmc_calib.hip "
                             "(profiles/r01_pmc/calibration_fetch_size.csv)",
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": (rd + wr) / alg,
        "launches": min(nf, nw),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (tools/gpu/pmc.sh running "
                  "tools/pmc_level0.py); Infinity-Cache hits are counted by these counters, so this is an upper "
                  "bound on HBM bytes",
    }
    dst.write_text(json.dumps(rec, indent=1))
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
