# every -m gpu test, then the 400^3 upload phase times (throughput mode, 3 cycles)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit $rc; }
SSS_HIP_TIMING=1 timeout -k 10 600 python -u tools/conv_study.py --n 400 --modes ${MODES:-throughput} --maxit 3 > gpurun_out/upload400.log 2>&1
rc=$?; grep "sss_hip\]\|iterations" gpurun_out/upload400.log; exit $rc
