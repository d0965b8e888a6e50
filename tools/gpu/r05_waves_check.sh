# fused engine with more waves in flight: GS tests, circuit and 7-pt 400^3 per-level pre-smoother times
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_engines.py > $O/wv_tests.log 2>&1 || { tail -30 $O/wv_tests.log; exit 1; }
tail -1 $O/wv_tests.log
timeout -k 10 300 python -u tools/gs_level_times.py --workload circuit --engines fused --reps 3 > $O/wv_circ.log 2>&1 || { tail -5 $O/wv_circ.log; exit 1; }
echo "circuit: $(grep '^\[gs\] fused' $O/wv_circ.log | awk '{print $3, $(NF-1)}' | tr '\n' ' ')"
timeout -k 10 900 python -u tools/gs_level_times.py --n 400 --engines fused --reps 3 > $O/wv_p400.log 2>&1 || { tail -5 $O/wv_p400.log; exit 1; }
echo "7pt400: $(grep '^\[gs\] fused' $O/wv_p400.log | awk '{print $3, $(NF-1)}' | tr '\n' ' ')"
