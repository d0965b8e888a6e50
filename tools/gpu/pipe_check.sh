# pipelined setup+upload: its GPU test, then the host phases of the default bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_setup_pipeline.py tests/test_gpu_free_order.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pipe_tests.log 2>&1
rc=$?; tail -12 gpurun_out/pipe_tests.log; [ $rc -eq 0 ] || exit $rc
HIPT=${HIPT:-1} bash tools/gpu/host_phases.sh
