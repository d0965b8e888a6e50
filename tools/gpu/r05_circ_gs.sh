# circuit stand-in: exact GS-CF pre-smoother per level, per-pass flow vs fused
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u tools/gs_level_times.py --workload circuit --engines flow,fused --reps 3 > $O/circ_gs.log 2>&1 || { tail -20 $O/circ_gs.log; exit 1; }
grep "^\[gs\]" $O/circ_gs.log
