# round 6: per-level exact GS-CF pre-smoother times at 400^3 with the fused engine (chain_fixed)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u tools/gs_level_times.py --n 400 --engines fused --reps 3 \
    --json $O/fused_levels_400.json > $O/fused_levels_400.log 2>&1 || { tail -20 $O/fused_levels_400.log; exit 1; }
grep "^\[gs\]" $O/fused_levels_400.log
