# round 6: the 27-pt 256^3 and circuit stand-in bench lines (throughput + parity mode) after chain_fixed
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/other
mkdir -p $O
timeout -k 10 500 python -u bench.py --stencil 27 --n 256 --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_a27_256.json 2> $O/bench_a27_256.err || { tail -20 $O/bench_a27_256.err; exit 1; }
timeout -k 10 400 python -u bench.py --workload circuit --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_circuit.json 2> $O/bench_circuit.err || { tail -20 $O/bench_circuit.err; exit 1; }
python - $O/bench_a27_256.json $O/bench_circuit.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    p = d.get("parity_mode", {})
    print(f.split("/")[-1], "throughput", round(d["value"], 2), "its", d["config"].get("iterations_to_tol"),
          "| parity", round(p.get("value", 0), 3), "V-cycles/s, its", p.get("iterations_to_tol"))
PY
