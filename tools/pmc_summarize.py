"""Level-0 SpMV HBM traffic from the two rocprofv3 --pmc passes of tools/gpu/pmc.sh.

    python tools/pmc_summarize.py gpurun_out profiles/r03_level0_spmv_pmc.json [commit]

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
import subprocess
import sys
from pathlib import Path

FETCH_CORRECTION = 2.0


def counter_avg(d: Path, name: str, csr: bool) -> tuple[float, int]:
    """launches of the level-0 residual: spmv_adaptive<2, false, 0> (CSR arrays) or the other
    instantiation (the cycle's storage)"""
    vals = []
    for f in d.rglob("*.csv"):
        with open(f) as fh:
            rd = csv.DictReader(fh)
            if "Counter_Name" not in (rd.fieldnames or []):
                continue
            for r in rd:
                kn = r["Kernel_Name"]
                if r["Counter_Name"] == name and "spmv_adaptive<2, false" in kn and \
                        ("spmv_adaptive<2, false, 0>" in kn) == csr:
                    vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {name} rows for the level-0 residual ({'CSR' if csr else 'stored'}) under {d}")
    return sum(vals) / len(vals), len(vals)


def main():
    out = Path(sys.argv[1])
    dst = Path(sys.argv[2])
    commit = sys.argv[3] if len(sys.argv) > 3 else None
    if commit is None:   # the tree that was sent to the box: this checkout's HEAD (+ "-dirty")
        try:
            commit = subprocess.run(["git", "describe", "--always", "--dirty"], capture_output=True, text=True,
                                    check=True).stdout.strip()
        except (OSError, subprocess.CalledProcessError):
            commit = "unknown"
    info = None
    for line in (out / "pmc_FETCH_SIZE.log").read_text().splitlines():
        if line.startswith("{"):
            info = json.loads(line)
    if info is None:
        raise SystemExit("pmc_level0.py JSON line not found")
    N, nnz = info["rows"], info["nnz"]
    survey = 12 * nnz + 4 * (N + 1) + 24 * N   # SURVEY.md 8(d), y = b - A x
    rec = {"n": info["n"], "rows": N, "nnz": nnz, "a_format": info["a_format"], "commit": commit}
    for key, csr, alg, ms in (("csr", True, survey, info.get("avg_ms_csr")),
                              ("stored", False, info["algorithmic_bytes_per_launch"], info["avg_ms"])):
        fetch, nf = counter_avg(out / "pmc_FETCH_SIZE", "FETCH_SIZE", csr)
        write, nw = counter_avg(out / "pmc_WRITE_SIZE", "WRITE_SIZE", csr)
        rd = fetch * 1024 * FETCH_CORRECTION
        wr = write * 1024
        rec[key] = {"kernel": "spmv_adaptive<RESID> level 0 from " + ("the CSR arrays" if csr else info["a_format"]),
                    "avg_ms_under_pmc_pass": ms, "fetch_size_kib_raw": fetch, "write_size_kib_raw": write,
                    "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                    "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes_per_launch": alg,
                    "traffic_over_algorithmic": (rd + wr) / alg, "launches": min(nf, nw)}
    rec.update({
        "fetch_correction": FETCH_CORRECTION,
        "correction_source": "MI355X_MICROARCH.md HBM section; re-measured with tools/pmc_calib.hip "
                             "(profiles/r01_pmc/calibration_fetch_size.csv)",
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (tools/gpu/pmc.sh running "
                  "tools/pmc_level0.py); Infinity-Cache hits are counted by these counters, so this is an upper "
                  "bound on HBM bytes",
    })
    dst.write_text(json.dumps(rec, indent=1))
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
