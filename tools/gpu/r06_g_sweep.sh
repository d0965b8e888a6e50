# round 6: lanes per row G on the fused engine's levels 1-6 at 400^3 after chain_fixed (fixed G per run)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/gsweep; mkdir -p $O
for g in ${GS:-4 8 16 32 64}; do
  SSS_HIP_FUSED_G=$g timeout -k 10 300 python -u tools/gs_level_times.py --n 400 --engines fused --reps 2 --levels ${LEVELS:-2,3,4,5,6} \
      > $O/G$g.log 2>&1 || { tail -5 $O/G$g.log; exit 1; }
  echo "G=$g"; grep "^\[gs\] fused" $O/G$g.log | awk '{print $3, $NF, $(NF-1)}' | tr '\n' ' '; echo
done
