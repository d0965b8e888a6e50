set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gs_engines.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gs_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gs_tests.log; exit 1; }
tail -3 gpurun_out/gs_tests.log
timeout -k 10 600 python -u tools/conv_study.py --n 256 --modes parity@cu,parity@flow,exact-direct --maxit 3 --json gpurun_out/conv256_gs.json > gpurun_out/conv256_gs.log 2>&1
grep "\[conv\]" gpurun_out/conv256_gs.log | tail -12
