# circuit stand-in and 7-pt 256^3: exact GS-CF pre-smoother per level, per-pass flow vs fused (G rule)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u tools/gs_level_times.py --workload circuit --engines flow,fused --reps 3 > $O/circ_gs2.log 2>&1 || { tail -20 $O/circ_gs2.log; exit 1; }
grep "^\[gs\]" $O/circ_gs2.log
timeout -k 10 600 python -u tools/gs_level_times.py --n 256 --levels 1,2,3 --engines fused --reps 3 > $O/p256_gs2.log 2>&1 || { tail -20 $O/p256_gs2.log; exit 1; }
grep "^\[gs\]" $O/p256_gs2.log
