# 7-pt 400^3 with stored-order sums everywhere (--sum-order 0): one GPU, then 8 ranks sharing it
# (host transport).  Every rank computes its rows from the same entries in the same order as one
# GPU, so the two relres histories agree to the norm's reduction order.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u bench.py --sum-order 0 --parity-cycles 0 --no-cpu-baseline --steps 5 --warmup 2 \
    > $O/bench_n1_400_so0.json 2> $O/bench_n1_400_so0.err || { tail -20 $O/bench_n1_400_so0.err; exit 1; }
timeout -k 10 900 python -u bench.py --gpus 8 --sum-order 0 --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/bench_g8_400_so0.json 2> $O/bench_g8_400_so0.err || { tail -20 $O/bench_g8_400_so0.err; exit 1; }
python3 - <<'PY'
import json
a = json.load(open("gpurun_out/r05/bench_n1_400_so0.json"))["config"]["relres_history"]
b = json.load(open("gpurun_out/r05/bench_g8_400_so0.json"))["config"]["relres_history"]
n = min(len(a), len(b))
print("iterations N=1", len(a), "N=8", len(b), "max rel diff", max(abs(x - y) / abs(x) for x, y in zip(a[:n], b[:n])))
PY
