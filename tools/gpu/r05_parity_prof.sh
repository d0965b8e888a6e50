# kernel-trace profile of the parity mode (exact GS-CF everywhere, device Krylov coarse solve) at 400^3
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
rm -rf $O/pprof
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/pprof -o run --output-format csv -- python3 bench.py --mode parity --steps 3 --warmup 1 --no-cpu-baseline --converge-max 0 --parity-cycles 0 > $O/pprof.log 2>&1 || { tail -30 $O/pprof.log; exit 1; }
grep '^{' $O/pprof.log | head -c 600; echo
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05/pprof/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.reader(open(f)))[1:]
tot = sum(float(r[2]) for r in rows)
rows.sort(key=lambda r: -float(r[2]))
for r in rows[:22]:
    print(f"{float(r[2])/tot*100:5.1f}% calls {r[1]:>6} avg {float(r[3])/1000:9.1f} us  {r[0][:100]}")
PY
