# Round 5 re-measurement at HEAD: the G3_circuit stand-in (bench line with its parity mirror to tol,
# then the kernel-trace profile and per-level split) and the 27-pt anisotropic 256^3 (bench line with
# the parity mirror to tol, then its kernel-trace profile)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 500 python -u bench.py --workload circuit --no-cpu-baseline > $O/bench_circ.json 2> $O/bench_circ.err || { tail -20 $O/bench_circ.err; exit 1; }
head -c 300 $O/bench_circ.json; echo
BENCH_ARGS="--workload circuit" bash tools/gpu/prof.sh > $O/prof_circ.out 2>&1 || { tail -20 $O/prof_circ.out; exit 1; }
cp gpurun_out/prof_levels.txt $O/circ_levels.txt; cp gpurun_out/prof_cur/run_kernel_stats.csv $O/circ_kernel_stats.csv
cat $O/circ_levels.txt
timeout -k 10 900 python -u bench.py --stencil 27 --n 256 --no-cpu-baseline > $O/bench_a27.json 2> $O/bench_a27.err || { tail -30 $O/bench_a27.err; exit 1; }
head -c 300 $O/bench_a27.json; echo
BENCH_ARGS="--stencil 27 --n 256" bash tools/gpu/prof.sh > $O/prof_a27.out 2>&1 || { tail -20 $O/prof_a27.out; exit 1; }
cp gpurun_out/prof_levels.txt $O/a27_levels.txt; cp gpurun_out/prof_cur/run_kernel_stats.csv $O/a27_kernel_stats.csv
cat $O/a27_levels.txt
