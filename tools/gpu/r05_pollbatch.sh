# fused engine: pending granules polled in batches -- GS + parity suites, level times, 400^3 parity trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gs_engines.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pollbatch_tests.log 2>&1 || { tail -40 $O/pollbatch_tests.log; exit 1; }
tail -2 $O/pollbatch_tests.log
timeout -k 10 240 python -u tools/gs_level_times.py --n 400 --levels 1,2,3,4,5,6 --engines fused --reps 3 > $O/p400_pollbatch.log 2>&1 || { tail -5 $O/p400_pollbatch.log; exit 1; }
echo "7pt400 pollbatch: $(grep '^\[gs\] fused' $O/p400_pollbatch.log | awk '{print $3, $(NF-1)}' | tr '\n' ' ')"
bash tools/gpu/r05_parity_prof.sh
