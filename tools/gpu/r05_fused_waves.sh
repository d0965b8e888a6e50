# lab: fused engine waves in flight (cap 1024 = 4 per CU today) on 256^3 levels 1-5
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 900 python -u tools/gs_level_times.py --n 256 --levels 1,2,3,4,5,8 --reps 3 \
    --engines fused,fused+SSS_LAB_FUSED_WAVES=2048,fused+SSS_LAB_FUSED_WMUL=8,fused+SSS_LAB_FUSED_WMUL=2 \
    > $O/fused_waves.log 2>&1 || { tail -20 $O/fused_waves.log; exit 1; }
grep "^\[gs\]" $O/fused_waves.log
