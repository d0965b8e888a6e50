# lab: fused engine, the chain overlapping the polls (default on rows >= 300) or after all pending resolved
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
SSS_HIP_TIMING=1 timeout -k 10 900 python -u tools/gs_level_times.py --n 400 --levels 4,5,6,7,8,9,10 --reps 3 \
    --engines fused,fused+SSS_LAB_FUSED_OVL=0,fused+SSS_LAB_FUSED_OVL=1 > $O/fovl_levels.log 2>&1 || { tail -20 $O/fovl_levels.log; exit 1; }
grep "fused GS-CF plan" $O/fovl_levels.log | head -8
grep "^\[gs\]" $O/fovl_levels.log | awk '{print $2, $3, $(NF-1)}'
