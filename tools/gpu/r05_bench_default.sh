# default bench at HEAD, summary line
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
T=${TAG:-head}
timeout -k 10 1000 python -u bench.py $BENCH_ARGS > $O/bench_$T.json 2> $O/bench_$T.log || { tail -30 $O/bench_$T.log; exit 1; }
python - "$O/bench_$T.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]; pm = d.get("parity_mode") or {}
print("value", round(d["value"], 3), "ms", round(d["ms_per_step"], 3), "setup", c.get("setup_s"), "upload", c.get("upload_s"),
      "its", c.get("iterations_to_tol"), "parity", pm.get("value"), "parity_upload", pm.get("upload_s"),
      "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
