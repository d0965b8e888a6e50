# exact GS-CF flow engine: per-level pre-smoother times at ${N:-256}^3 for the default and each
# "VAR=value" of $KNOBS (tools/gs_level_times.py)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gs_level_times.py --n ${N:-256} --engines flow --reps 3 > gpurun_out/gsk_base.txt 2>&1 || { tail -20 gpurun_out/gsk_base.txt; exit 1; }
echo "== base"; grep "\[gs\]" gpurun_out/gsk_base.txt
for kv in $KNOBS; do
  t=$(echo "$kv" | tr "/" "_")
  env "$kv" timeout -k 10 300 python -u tools/gs_level_times.py --n ${N:-256} --engines flow --reps 3 > "gpurun_out/gsk_$t.txt" 2>&1 || { tail -20 "gpurun_out/gsk_$t.txt"; exit 1; }
  echo "== $kv"; grep "\[gs\]" "gpurun_out/gsk_$t.txt"
done
