# the other BASELINE workloads on one GPU at HEAD: G3_circuit stand-in and 27-pt anisotropic 256^3 bench
# lines, each with a kernel-trace profile split per level
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload circuit --no-cpu-baseline > gpurun_out/bench_circuit.json 2> gpurun_out/bench_circuit.err || { tail -20 gpurun_out/bench_circuit.err; exit 1; }
head -c 300 gpurun_out/bench_circuit.json; echo
BENCH_ARGS="--workload circuit" bash tools/gpu/prof.sh > /dev/null && cp gpurun_out/prof_levels.txt gpurun_out/circuit_levels.txt
tail -14 gpurun_out/circuit_levels.txt
timeout -k 10 900 python -u bench.py --stencil 27 --n 256 --no-cpu-baseline --parity-cycles 0 > gpurun_out/bench_a27.json 2> gpurun_out/bench_a27.err || { tail -20 gpurun_out/bench_a27.err; exit 1; }
head -c 300 gpurun_out/bench_a27.json; echo
