# round 6 evidence, lease 2: kernel-trace profile of a short default bench with its per-level split,
# the roctx ranges (marker trace, its own run: never combined with --pmc), the SQ occupancy / stall pass
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06/evidence
mkdir -p $O
bash tools/gpu/prof.sh > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
tail -16 gpurun_out/prof_levels.txt
f=$(find gpurun_out/prof_cur -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats.csv
cp gpurun_out/prof_levels.txt gpurun_out/prof_bench.json $O/
rm -rf gpurun_out/prof_cur
rm -rf gpurun_out/marker
timeout -k 10 600 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/marker -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --converge-max 0 --parity-cycles 1 --parity-converge 0 \
    > $O/marker.log 2>&1 || { tail -20 $O/marker.log; exit 1; }
m=$(find gpurun_out/marker -name '*marker_api_trace.csv' | head -1)
python3 - "$m" > $O/roctx_ranges.txt <<'PY'
import csv, sys
from collections import defaultdict
tot = defaultdict(float); cnt = defaultdict(int)
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get("Function") or r.get("Name") or r.get("Message") or ""
    try:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    except Exception:
        continue
    tot[n] += d; cnt[n] += 1
print(f"{'roctx range':50s} {'count':>6s} {'total ms':>10s}")
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:60]:
    print(f"{n[:50]:50s} {cnt[n]:6d} {t:10.2f}")
PY
head -25 $O/roctx_ranges.txt
rm -rf gpurun_out/marker
bash tools/gpu/pmc_sq.sh > $O/pmc_sq.out 2>&1 || { tail -20 $O/pmc_sq.out; exit 1; }
cp gpurun_out/kernels_sq_pmc.txt $O/
head -12 $O/kernels_sq_pmc.txt
