# lab: fused engine waves in flight on the long-row levels of 400^3 (32 today: 4 per depth chunk, min 32)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 900 python -u tools/gs_level_times.py --n 400 --reps 3 \
    --levels 2,3,4,5,6,8,10 --engines fused+SSS_LAB_FUSED_WMIN=512,fused+SSS_LAB_FUSED_WMIN=1024,fused+SSS_LAB_FUSED_WMIN=2048+SSS_LAB_FUSED_WCAP=2048 > $O/fw2_levels.log 2>&1 || { tail -20 $O/fw2_levels.log; exit 1; }
grep "^\[gs\]" $O/fw2_levels.log | awk '{print $2, $3, $(NF-1)}'
