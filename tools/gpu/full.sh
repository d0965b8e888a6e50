# Whole GPU check: every -m gpu test, 256^3 parity/throughput histories, default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$CONV" ]; then
timeout -k 10 600 python -u tools/conv_study.py --n 256 --modes $CONV --maxit 40 --json gpurun_out/conv256.json > gpurun_out/conv256.log 2>&1
rc=$?; grep "\[conv\].*iterations" gpurun_out/conv256.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
timeout -k 10 900 python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.err; exit $rc; }
fi
