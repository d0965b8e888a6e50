"""L2 behaviour per kernel launch shape from one rocprofv3 --pmc pass (tools/gpu/pmc_l2.sh):
TCC_HIT_sum, TCC_MISS_sum (L2 hits / misses, all XCDs) and TCP_TCC_READ_REQ_sum (L1 -> L2 read
requests), averaged over the launches of each (kernel, workgroups) shape -- one template serves every
level, the workgroup count tells the levels apart.

    python tools/pmc_levels.py gpurun_out/pmc_l2 > profiles/r02_levels_l2_pmc.txt
"""
import collections
import csv
import sys
from pathlib import Path


def main():
    d = Path(sys.argv[1])
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in d.rglob("*.csv"):
        with open(f) as fh:
            rd = csv.DictReader(fh)
            if "Counter_Name" not in (rd.fieldnames or []):
                continue
            for r in rd:
                wg = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
                key = (r["Kernel_Name"].split("(")[0][:48], wg)
                acc[key][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    rows = []
    for key, per in acc.items():
        disp = collections.defaultdict(dict)
        for (did, cn), v in per.items():
            disp[did][cn] = sum(v)
        n = len(disp)
        hit = sum(x.get("TCC_HIT_sum", 0) for x in disp.values()) / n
        miss = sum(x.get("TCC_MISS_sum", 0) for x in disp.values()) / n
        req = sum(x.get("TCP_TCC_READ_REQ_sum", 0) for x in disp.values()) / n
        rows.append((hit + miss, key, n, hit, miss, req))
    rows.sort(reverse=True)
    print(f"{'kernel':50s} {'WGs':>8s} {'calls':>5s} {'L2 hit':>12s} {'L2 miss':>12s} {'hit %':>6s} {'L1->L2 rd':>12s}")
    for _, (k, wg), n, hit, miss, req in rows[:40]:
        print(f"{k:50s} {wg:8d} {n:5d} {hit:12.0f} {miss:12.0f} {100 * hit / max(hit + miss, 1):6.1f} {req:12.0f}")


if __name__ == "__main__":
    main()
