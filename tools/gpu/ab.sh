# A/B of engine variants on the per-level kernel times of the bench workload (kernel-trace profile
# of a short bench per variant).  Variants: label=ENV=VAL[,ENV=VAL...] arguments, e.g.
#   bash tools/gpu/ab.sh head= prev=SSS_AMG_LIB=amg_amd/lib_ab/libsss_amg.so nodict=SSS_HIP_DICT=0
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
for v in "$@"; do
    label=${v%%=*}; envs=${v#*=}
    ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
      [ -n "$SSS_AMG_LIB" ] && export SSS_AMG_LIB="$GRAFT_REPO_ROOT/${SSS_AMG_LIB#$GRAFT_REPO_ROOT/}"
      bash tools/gpu/prof.sh > gpurun_out/ab/$label.out 2>&1 ) || { echo "variant $label failed"; tail -20 gpurun_out/ab/$label.out; exit 1; }
    cp gpurun_out/prof_levels.txt gpurun_out/ab/levels_$label.txt
    cp gpurun_out/prof_bench.json gpurun_out/ab/bench_$label.json
    echo "== $label: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/bench_$label.json)"
    tail -4 gpurun_out/ab/levels_$label.txt
done
rm -rf gpurun_out/prof_cur
