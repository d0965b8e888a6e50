# A/B of per-level kernel times: the default, then each "VAR=value" given in $AB (space-separated)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
bash tools/gpu/prof.sh > gpurun_out/ab/base.out 2>&1 || { tail -20 gpurun_out/ab/base.out; exit 1; }
cp gpurun_out/prof_levels.txt gpurun_out/ab/base_levels.txt
cp gpurun_out/prof_bench.json gpurun_out/ab/base_bench.json
echo "== base"; cat gpurun_out/ab/base_levels.txt
python3 -c "import json,sys; r=json.load(open(sys.argv[1]))['roofline']; print('roofline ms', r['avg_launch_ms'], 'cycle_storage ms', r['cycle_storage']['avg_launch_ms'])" gpurun_out/ab/base_bench.json
for kv in $AB; do
  t=$(echo "$kv" | tr "/" "_")
  env "$kv" bash tools/gpu/prof.sh > "gpurun_out/ab/$t.out" 2>&1 || { tail -20 "gpurun_out/ab/$t.out"; exit 1; }
  cp gpurun_out/prof_levels.txt "gpurun_out/ab/${t}_levels.txt"
  cp gpurun_out/prof_bench.json "gpurun_out/ab/${t}_bench.json"
  echo "== $kv"; cat "gpurun_out/ab/${t}_levels.txt"
  python3 -c "import json,sys; r=json.load(open(sys.argv[1]))['roofline']; print('roofline ms', r['avg_launch_ms'], 'cycle_storage ms', r['cycle_storage']['avg_launch_ms'])" "gpurun_out/ab/${t}_bench.json"
done
