# a subset of the -m gpu tests: bash tools/gpu/tests_subset.sh tests/test_a.py tests/test_b.py ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_subset.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_subset.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/gpu_subset.log | head -30; exit $rc; }
