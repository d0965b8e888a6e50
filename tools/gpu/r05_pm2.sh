# fused-engine tests, then the parity mirror phases at 400^3
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_engines.py \
    > $O/pm2_tests.log 2>&1 || { tail -30 $O/pm2_tests.log; exit 1; }
tail -1 $O/pm2_tests.log
SSS_HIP_TIMING=2 timeout -k 10 400 python -u tools/parity_mirror_time.py --n 400 > $O/pm2_phases.log 2>&1 || { tail -20 $O/pm2_phases.log; exit 1; }
grep -E "\[pm\]" $O/pm2_phases.log
