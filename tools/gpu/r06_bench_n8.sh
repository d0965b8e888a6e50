# round 6: bench.py at N = 1 and N = 8 (8 ranks sharing the one GPU, host transport) with stored-order
# sums, so the two relres histories can be compared (BASELINE.json configs[2] at --n 512)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/bench_n8
mkdir -p "$O"
N=${N:-400}
timeout -k 10 500 python -u bench.py --n $N --sum-order 0 --no-cpu-baseline --parity-cycles 0 --steps 3 --warmup 1 \
    > "$O/n1_${N}_sumorder0.json" 2> "$O/n1_${N}_sumorder0.err"
rc=$?; cat "$O/n1_${N}_sumorder0.json" | head -c 600; echo; [ $rc -eq 0 ] || { tail -20 "$O/n1_${N}_sumorder0.err"; exit $rc; }
timeout -k 10 ${N8_LIMIT:-700} python -u bench.py --gpus 8 --n $N --sum-order 0 --no-cpu-baseline --steps 3 --warmup 1 \
    > "$O/n8_${N}_sumorder0.json" 2> "$O/n8_${N}_sumorder0.err"
rc=$?; cat "$O/n8_${N}_sumorder0.json" | head -c 600; echo; [ $rc -eq 0 ] || tail -20 "$O/n8_${N}_sumorder0.err"; exit $rc
