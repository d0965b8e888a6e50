# round 6: fused GS engine waves in flight (SSS_HIP_FUSED_WAVES) on the long-row levels at 400^3
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/waves; mkdir -p $O
for w in ${WS:-256 512 1024 2048}; do
  SSS_HIP_FUSED_WAVES=$w timeout -k 10 300 python -u tools/gs_level_times.py --n 400 --engines fused --reps 2 --levels 5,6,7,8,9 \
      > $O/W$w.log 2>&1 || { tail -5 $O/W$w.log; exit 1; }
  echo "waves=$w $(grep '^\[gs\] fused' $O/W$w.log | awk '{print $3, $NF}' | tr '\n' ' ')"
done
