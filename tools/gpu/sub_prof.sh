# the GPU tests of the tile/ELL kernels (parity, engines, distributed), then prof.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gs_engines.py tests/test_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit $rc; }
bash tools/gpu/prof.sh
