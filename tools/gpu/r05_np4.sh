# lab: fused engine polls per lane and round (NP = 4 instead of 2): tests, 400^3 level times, default bench
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_engines.py > $O/np4_tests.log 2>&1 || { tail -30 $O/np4_tests.log; exit 1; }
tail -1 $O/np4_tests.log
timeout -k 10 900 python -u tools/gs_level_times.py --n 400 --levels 5,6,7,8,9,10 --engines fused --reps 3 > $O/np4_levels.log 2>&1 || { tail -5 $O/np4_levels.log; exit 1; }
echo "np4: $(grep '^\[gs\] fused' $O/np4_levels.log | awk '{print $3, $(NF-1)}' | tr '\n' ' ')"
