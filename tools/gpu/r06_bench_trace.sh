# round 6: smoke(), then the default bench line with the one-launch CG's phase trace on stderr
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/${TAG:-bench_trace}
mkdir -p "$O"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
rc=$?; tail -2 "$O/smoke.log"; [ $rc -eq 0 ] || exit $rc
SSS_HIP_CG_TRACE=1 timeout -k 10 700 python -u bench.py ${BENCH_ARGS} > "$O/bench.json" 2> "$O/bench.err"
rc=$?; grep "cg trace" "$O/bench.err" | head -3; [ $rc -eq 0 ] || { tail -20 "$O/bench.err"; exit $rc; }
python - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d.get("parity_mode", {})
print("headline", d["value"], d["unit"], "ms/step", d["ms_per_step"], "| parity ms/cycle", p.get("ms_per_step"),
      "| roofline", d.get("roofline", {}).get("frac"), "| cpu", d.get("cpu_baseline", {}).get("value"))
PY
