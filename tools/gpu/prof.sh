# kernel-trace profile of a short bench run (N=1) + per-level breakdown of one V-cycle
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_cur
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cur -o run --output-format rocpd csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --converge-max 0 --parity-cycles 0 ${BENCH_ARGS} > gpurun_out/prof_cur.log 2>&1 || { echo prof failed; tail -30 gpurun_out/prof_cur.log; exit 1; }
grep '^{' gpurun_out/prof_cur.log > gpurun_out/prof_bench.json
python3 tools/level_breakdown.py $(find gpurun_out/prof_cur -name '*.db' | head -1) gpurun_out/prof_bench.json | tee gpurun_out/prof_levels.txt
# per (kernel, workgroups): the level-0 launches of the roofline kernel apart from the other levels'
python3 tools/prof_summary.py $(find gpurun_out/prof_cur -name '*.db' | head -1) --shapes gpurun_out/prof_shapes.txt > /dev/null
