# round 6: the new GPU tests first (host-entry zero iterate and stall, SuiteSparse harness), a
# rehearsal of the 8-rank harness at 128^3, then BASELINE configs[2] at 512^3 over 8 ranks
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/new_tests
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_gs_engines.py tests/test_gpu_suitesparse.py -m gpu -x -v \
    -k "zero_iterate or stall or suitesparse or mtx" --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" "$O/tests.log" | head -30; exit $rc; }
SSS_TEST_DIST_N=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_512.py -m gpu -x -v --timeout 280 \
    --timeout-method thread > "$O/dist128.log" 2>&1
rc=$?; tail -3 "$O/dist128.log"; cp gpurun_out/test_dist_512.log "$O/dist128_helper.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 850 python -u -m pytest tests/test_gpu_dist_512.py -m gpu -x -v --timeout 840 \
    --timeout-method thread > "$O/dist512.log" 2>&1
rc=$?; tail -3 "$O/dist512.log"; cp gpurun_out/test_dist_512.log "$O/dist512_helper.log"; exit $rc
