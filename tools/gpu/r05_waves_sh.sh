# fused engine with sharded tickets: waves in flight 1024 / 1536 / 2048, 7-pt 400^3 levels 1-6 at the planned G
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
for w in 1024 1536 2048; do
  SSS_HIP_FUSED_WAVES=$w timeout -k 10 240 python -u tools/gs_level_times.py --n 400 --levels 1,2,3,4,5,6 --engines fused --reps 3 > $O/p400_waves$w.log 2>&1 || { tail -5 $O/p400_waves$w.log; exit 1; }
  echo "7pt400 waves=$w: $(grep '^\[gs\] fused' $O/p400_waves$w.log | awk '{print $3, $(NF-1)}' | tr '\n' ' ')"
done
