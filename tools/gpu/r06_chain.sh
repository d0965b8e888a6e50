# round 6: the fixed-schedule in-order chain (chain_fixed) in the GS engines and the one-launch coarse
# CG -- the GS-engine and parity GPU tests (bitwise), then the default bench (headline + parity mode)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/chain
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_gs_engines.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" "$O/tests.log" | head -30; exit $rc; }
SSS_HIP_CG_TRACE=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; grep "cg trace" "$O/bench.err" | head -2; [ $rc -eq 0 ] || { tail -20 "$O/bench.err"; exit $rc; }
python - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d.get("parity_mode", {})
print("headline", d["value"], d["unit"], "ms/step", d["ms_per_step"], "| parity ms/cycle", p.get("ms_per_step"))
PY
