set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_dist_gpu.py -x -q > gpurun_out/dist_tests.log 2>&1 || { echo "dist pytest failed"; tail -60 gpurun_out/dist_tests.log; exit 1; }
echo dist-ok
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
echo tests-ok
