# lab: fused engine lanes per row (G) and chunks per ticket on the short-row levels (256^3 and 400^3 L1-L3)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
SSS_LAB_FUSED_G=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_engines.py -k "fused" \
    > $O/fused_g_tests.log 2>&1 || { tail -30 $O/fused_g_tests.log; exit 1; }
tail -1 $O/fused_g_tests.log
timeout -k 10 900 python -u tools/gs_level_times.py --n 256 --levels 1,2 --reps 3 \
    --engines fused+SSS_LAB_FUSED_G=1,fused+SSS_LAB_FUSED_G=2,fused+SSS_LAB_FUSED_G=4 \
    > $O/fused_g.log 2>&1 || { tail -20 $O/fused_g.log; exit 1; }
grep "^\[gs\]" $O/fused_g.log
