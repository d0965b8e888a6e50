# every -m gpu test, then the per-level kernel profile of the bench workload (prof.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit $rc; }
bash tools/gpu/prof.sh
