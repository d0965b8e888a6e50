# after restoring the G = 4 kernel: GS engine tests, then circuit and 7-pt per-level fused times
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_engines.py > $O/g4_tests.log 2>&1 || { tail -30 $O/g4_tests.log; exit 1; }
tail -1 $O/g4_tests.log
for g in 4 8 16; do
  SSS_HIP_FUSED_G=$g timeout -k 10 200 python -u tools/gs_level_times.py --workload circuit --engines fused --reps 3 > $O/circ_g$g.log 2>&1 || { tail -5 $O/circ_g$g.log; exit 1; }
  echo "circuit G=$g: $(grep '^\[gs\] fused' $O/circ_g$g.log | awk '{print $3, $(NF-1)}' | tr '\n' ' ')"
done
timeout -k 10 200 python -u tools/gs_level_times.py --workload circuit --engines fused --reps 3 > $O/circ_rule.log 2>&1 || { tail -5 $O/circ_rule.log; exit 1; }
echo "circuit rule: $(grep '^\[gs\] fused' $O/circ_rule.log | awk '{print $3, $(NF-1)}' | tr '\n' ' ')"
