# lanes-per-row rule: plans and per-level fused times on the circuit stand-in and 7-pt 256^3
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
SSS_HIP_TIMING=1 timeout -k 10 200 python -u tools/gs_level_times.py --workload circuit --engines fused --reps 3 > $O/circ_grule.log 2>&1 || { tail -5 $O/circ_grule.log; exit 1; }
grep "fused GS-CF plan" $O/circ_grule.log
echo "circuit rule: $(grep '^\[gs\] fused' $O/circ_grule.log | awk '{print $3, $(NF-1)}' | tr '\n' ' ')"
SSS_HIP_TIMING=1 timeout -k 10 300 python -u tools/gs_level_times.py --n 256 --engines fused --reps 3 > $O/p256_grule.log 2>&1 || { tail -5 $O/p256_grule.log; exit 1; }
grep "fused GS-CF plan" $O/p256_grule.log
echo "7pt256 rule: $(grep '^\[gs\] fused' $O/p256_grule.log | awk '{print $3, $(NF-1)}' | tr '\n' ' ')"
