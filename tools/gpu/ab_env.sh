# A/B of per-level kernel times: the default, then each "VAR=value" given in $AB (space-separated)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
bash tools/gpu/prof.sh > gpurun_out/ab/base.out 2>&1 || { tail -20 gpurun_out/ab/base.out; exit 1; }
cp gpurun_out/prof_levels.txt gpurun_out/ab/base_levels.txt
echo "== base"; cat gpurun_out/ab/base_levels.txt
for kv in $AB; do
  env "$kv" bash tools/gpu/prof.sh > "gpurun_out/ab/$kv.out" 2>&1 || { tail -20 "gpurun_out/ab/$kv.out"; exit 1; }
  cp gpurun_out/prof_levels.txt "gpurun_out/ab/${kv}_levels.txt"
  echo "== $kv"; cat "gpurun_out/ab/${kv}_levels.txt"
done
