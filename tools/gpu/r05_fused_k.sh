# lab: fused engine chunks per ticket (ticket-atomic throughput) on 256^3 levels; bitwise suite with K=4
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
SSS_LAB_FUSED_K=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_engines.py \
    > $O/fused_k_tests.log 2>&1 || { tail -30 $O/fused_k_tests.log; exit 1; }
tail -1 $O/fused_k_tests.log
timeout -k 10 900 python -u tools/gs_level_times.py --n 256 --levels 1,2,3,4,5,8 --reps 3 \
    --engines fused,fused+SSS_LAB_FUSED_K=2,fused+SSS_LAB_FUSED_K=4,fused+SSS_LAB_FUSED_K=8 \
    > $O/fused_k.log 2>&1 || { tail -20 $O/fused_k.log; exit 1; }
grep "^\[gs\]" $O/fused_k.log
