# lab: which fused configuration stalls on the circuit stand-in's level 1
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
for cfg in "G=2 D=host" "G=4 D=host" "G=4 D=gpu" "G=8 D=host" "G=16 D=host"; do
  g=${cfg#G=}; g=${g%% *}; d=${cfg##*D=}
  SSS_LAB_FUSED_G=$g SSS_HIP_FUSED_DEPTH=$d timeout -k 10 120 python -u tools/gs_level_times.py --workload circuit --levels 1,2,8 --engines fused --reps 2 > $O/circ_stall_$g$d.log 2>&1
  echo "$cfg rc=$? $(grep -c '^\[gs\] fused' $O/circ_stall_$g$d.log) $(grep '^\[gs\] fused' $O/circ_stall_$g$d.log | awk '{print $3, $NF-0, $(NF-1)}' | tr '\n' ' ')"
done
