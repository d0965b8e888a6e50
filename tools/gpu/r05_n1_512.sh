# 7-pt 512^3 on one GPU: throughput mode to tol and the parity (reference-semantics) mirror to tol in
# the same run -- the reference iteration count at BASELINE.json configs[2]'s problem size
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 1100 python -u bench.py --n 512 --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/bench_n1_512.json 2> $O/bench_n1_512.err || { echo "bench n1 512 failed rc=$?"; tail -30 $O/bench_n1_512.err; exit 1; }
head -c 1200 $O/bench_n1_512.json; echo
