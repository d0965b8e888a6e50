# One-launch exact GS engines: GPU tests, then 256^3 parity-mode V-cycle times per engine.
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_gs_engines.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gs_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gs_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/conv_study.py --n 256 --modes ${GS_MODES:-parity@cu,parity@flow,parity} --maxit ${GS_MAXIT:-3} --json gpurun_out/conv256_gs.json > gpurun_out/conv256_gs.log 2>&1
rc=$?
grep "\[conv\]" gpurun_out/conv256_gs.log
exit $rc
