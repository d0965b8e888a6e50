# round 6: chain_fixed's 8-wide tail -- GS-engine + parity GPU tests, per-level fused GS times, parity cycle
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/chain2
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_gs_engines.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; tail -2 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" "$O/tests.log" | head -30; exit $rc; }
timeout -k 10 600 python -u tools/gs_level_times.py --n 400 --engines fused --reps 3 --json $O/fused_levels_400.json \
    > $O/fused_levels_400.log 2>&1 || { tail -20 $O/fused_levels_400.log; exit 1; }
grep "^\[gs\]" $O/fused_levels_400.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --parity-cycles 3 --parity-converge 0 --converge-max 0 --steps 2 \
    --warmup 1 > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('parity ms/cycle', d['parity_mode']['ms_per_step'], 'headline', d['value'])" "$O/bench.json"
