# round 5: fused exact GS-CF engine -- bitwise suite, then per-level smoother times (flow vs fused)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_engines.py \
    > $O/fused_tests.log 2>&1 || { tail -30 $O/fused_tests.log; exit 1; }
tail -3 $O/fused_tests.log
timeout -k 10 500 python -u tools/gs_level_times.py --n ${N:-256} --engines flow,fused --reps 3 \
    --json $O/fused_levels_${N:-256}.json > $O/fused_levels_${N:-256}.log 2>&1 || { tail -20 $O/fused_levels_${N:-256}.log; exit 1; }
grep "^\[gs\]" $O/fused_levels_${N:-256}.log
