# round 6: every -m gpu test (or $TESTS), then smoke() and the default bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06
O=gpurun_out/r06/${TAG:-suite}
mkdir -p "$O"
timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
rc=$?; tail -3 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" "$O/gpu_tests.log" | head -30; exit $rc; }
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
rc=$?; tail -2 "$O/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > "$O/bench.json" 2> "$O/bench.err"
rc=$?; cat "$O/bench.json"; [ $rc -eq 0 ] || tail -20 "$O/bench.err"; exit $rc
