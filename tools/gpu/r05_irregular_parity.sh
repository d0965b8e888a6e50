# circuit stand-in and 27-pt 256^3 bench lines at HEAD (parity mirrors to tol on the fused GS-CF engine)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 500 python -u bench.py --workload circuit --no-cpu-baseline > $O/bench_circ_fused.json 2> $O/bench_circ_fused.err || { tail -20 $O/bench_circ_fused.err; exit 1; }
timeout -k 10 900 python -u bench.py --stencil 27 --n 256 --no-cpu-baseline > $O/bench_a27_fused.json 2> $O/bench_a27_fused.err || { tail -30 $O/bench_a27_fused.err; exit 1; }
for f in circ_fused a27_fused; do
python - "$O/bench_$f.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]; pm = d.get("parity_mode") or {}
print(c.get("workload"), "value", round(d["value"], 2), "its", c.get("iterations_to_tol"), "parity", pm.get("value"),
      "parity_its", pm.get("iterations_to_tol"), "engines", pm.get("gs_engines"), "upload", pm.get("upload_s"))
PY
done
