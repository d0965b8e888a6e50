# fused engine with the GPU-built depth and hashed symmetry checks: bitwise suite, parity mirror phases at 400^3
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_engines.py \
    > $O/fused2_tests.log 2>&1 || { tail -30 $O/fused2_tests.log; exit 1; }
tail -2 $O/fused2_tests.log
SSS_HIP_TIMING=2 timeout -k 10 400 python -u tools/parity_mirror_time.py --n 400 > $O/fused2_mirror400.log 2>&1 || { tail -20 $O/fused2_mirror400.log; exit 1; }
grep -E "smoother plan|\[pm\]" $O/fused2_mirror400.log | tail -30
