# GS engine tests, then per-level exact GS-CF smoother times per engine (tools/gs_level_times.py)
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_gs_engines.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gs_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gs_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/gs_level_times.py --n ${GS_N:-256} --engines ${GS_ENGINES:-launch,flow,flow:64,flow:512,cu} --json gpurun_out/gs_levels.json > gpurun_out/gs_levels.log 2>&1
rc=$?
grep "\[gs\]" gpurun_out/gs_levels.log
exit $rc
