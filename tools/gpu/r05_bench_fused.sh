# default bench at HEAD (parity mode now on the fused exact GS-CF engine), mirror phases in the log
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
SSS_HIP_TIMING=1 timeout -k 10 1000 python -u bench.py > $O/bench_fused.json 2> $O/bench_fused.log || { tail -30 $O/bench_fused.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05/bench_fused.json").read().strip().splitlines()[-1])
pm = d.get("parity_mode", {})
print("value", d["value"], "ms", d["ms_per_step"], "parity", {k: pm.get(k) for k in ("value", "upload_s", "ms_per_cycle")},
      "cpu", d["cpu_baseline"]["value"], "setup", d.get("setup_s"), d.get("upload_s"))
PY
