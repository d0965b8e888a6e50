# fused engine lanes per row with sharded tickets on 7-pt 400^3 levels 1-5 (2-sweep pre-smoother per level)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
for g in 2 4 8 16 32 64; do
  SSS_HIP_FUSED_G=$g timeout -k 10 240 python -u tools/gs_level_times.py --n 400 --levels 1,2,3,4,5 --engines fused --reps 3 > $O/p400_sh_g$g.log 2>&1 || { tail -5 $O/p400_sh_g$g.log; exit 1; }
  echo "7pt400 G=$g: $(grep '^\[gs\] fused' $O/p400_sh_g$g.log | awk '{print $3, $(NF-1)}' | tr '\n' ' ')"
done
