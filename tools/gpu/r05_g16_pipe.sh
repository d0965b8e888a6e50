# lab: fused engine with 16-byte granules and/or pipelined polls -- bitwise suite, then 400^3 levels 5-10
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
SSS_LAB_G16=1 SSS_LAB_PIPE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_engines.py > $O/g16p_tests.log 2>&1 || { tail -30 $O/g16p_tests.log; exit 1; }
tail -1 $O/g16p_tests.log
timeout -k 10 900 python -u tools/gs_level_times.py --n 400 --levels 2,5,6,7,8,9,10 --reps 3 \
    --engines fused,fused+SSS_LAB_G16=1,fused+SSS_LAB_PIPE=1,fused+SSS_LAB_G16=1+SSS_LAB_PIPE=1 > $O/g16p_levels.log 2>&1 || { tail -20 $O/g16p_levels.log; exit 1; }
grep "^\[gs\]" $O/g16p_levels.log | awk '{print $2, $3, $(NF-1)}'
