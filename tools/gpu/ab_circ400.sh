cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/prof.sh > gpurun_out/prof.out 2>&1 || { tail -20 gpurun_out/prof.out; exit 1; }
cp gpurun_out/prof_levels.txt gpurun_out/prof_levels_400.txt; cp gpurun_out/prof_bench.json gpurun_out/prof_bench_400.json
timeout -k 10 400 python -u bench.py --workload circuit --no-cpu-baseline > gpurun_out/bench_circ.json 2> gpurun_out/bench_circ.err || { tail -20 gpurun_out/bench_circ.err; exit 1; }
head -c 300 gpurun_out/bench_circ.json; echo
tail -17 gpurun_out/prof_levels_400.txt
