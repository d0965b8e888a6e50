# round 6: the one-launch CG with 1, 2 or 4 chaining waves per SIMD (SSS_HIP_CG_CHAINERS): trace + parity cycle
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/chainers; mkdir -p $O
for c in ${CS:-1 2 4}; do
  SSS_HIP_CG_CHAINERS=$c SSS_HIP_CG_TRACE=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --parity-cycles 3 \
      --parity-converge 0 --converge-max 0 --steps 2 --warmup 1 > $O/b$c.json 2> $O/b$c.err || { tail -5 $O/b$c.err; exit 1; }
  echo "chainers $c: $(grep 'cg trace' $O/b$c.err | head -1 | cut -c1-230)"
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('  parity ms/cycle', d['parity_mode']['ms_per_step'])" $O/b$c.json
done
