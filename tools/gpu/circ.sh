# circuit workload: its GPU tests, the free-order/parity suites the changes touch, a bench line
# and a per-level kernel profile
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -s --timeout 500 --timeout-method thread -m gpu > gpurun_out/tc.log 2>&1
rc=$?; grep -E "circuit 1.58M|passed|failed|FAIL|Error" gpurun_out/tc.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload circuit > gpurun_out/bench_circ.json 2> gpurun_out/bench_circ.err || { tail -20 gpurun_out/bench_circ.err; exit 1; }
cat gpurun_out/bench_circ.json
BENCH_ARGS="--workload circuit" bash tools/gpu/prof.sh
