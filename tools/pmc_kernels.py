"""Per-kernel-shape averages of every counter of one rocprofv3 --pmc pass (any counter set).

    python tools/pmc_kernels.py gpurun_out/pmc_sq [top]

One template serves every level, so launches are grouped by (kernel, workgroups).  Derived columns
for the SQ set of tools/gpu/pmc_sq.sh: waves per launch, busy fraction of the wave cycles
(ACTIVE_INST / WAVE_CYCLES), stalled-on-memory fraction (WAIT_ANY / WAVE_CYCLES), issue-stall
fraction (WAIT_INST_ANY / WAVE_CYCLES), vector-memory reads per wave, and the mean waves resident
per CU (WAVE_CYCLES quad-cycles x 4 / GRBM_GUI_ACTIVE cycles / 256 CUs; GRBM_GUI_ACTIVE is summed
over the 8 XCDs, so / 8 per XCD clock -- MI355X_MICROARCH.md, rocprofv3 PMC slots and DVFS).
"""
import collections
import csv
import sys
from pathlib import Path


def main():
    d = Path(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    names = set()
    for f in d.rglob("*.csv"):
        with open(f) as fh:
            rd = csv.DictReader(fh)
            if "Counter_Name" not in (rd.fieldnames or []):
                continue
            for r in rd:
                wg = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
                key = (r["Kernel_Name"].split("(")[0].replace("void ", "")[:44], wg)
                acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
                calls[key].add(r["Dispatch_Id"])
                names.add(r["Counter_Name"])
    rows = []
    for key, c in acc.items():
        n = len(calls[key])
        rows.append((c.get("SQ_WAVE_CYCLES", c.get("GRBM_GUI_ACTIVE", 0)), key, n, {k: v / n for k, v in c.items()}))
    rows.sort(reverse=True)
    print(f"{'kernel':44s} {'WGs':>7s} {'n':>3s} {'waves':>8s} {'active':>6s} {'waitmem':>7s} {'waitins':>7s} "
          f"{'vmem/wv':>7s} {'occ/CU':>6s} {'gui_us':>7s}")
    for _, (k, wg), n, c in rows[:top]:
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        waves = c.get("SQ_WAVES", 0.0)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0   # per-XCD cycles
        fr = lambda x: (100.0 * c.get(x, 0.0) / wc) if wc else 0.0   # noqa: E731
        occ = (4.0 * wc / gui / 256.0) if gui else 0.0
        vm = c.get("SQ_INSTS_VMEM_RD", 0.0) / waves if waves else 0.0
        print(f"{k:44s} {wg:7d} {n:3d} {waves:8.0f} {fr('SQ_ACTIVE_INST_ANY'):6.1f} {fr('SQ_WAIT_ANY'):7.1f} "
              f"{fr('SQ_WAIT_INST_ANY'):7.1f} {vm:7.1f} {occ:6.1f} {gui / 2400.0:7.1f}")
    print("counters:", ", ".join(sorted(names)))


if __name__ == "__main__":
    main()
