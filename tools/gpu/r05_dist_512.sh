# Round 5: BASELINE.json configs[2] (7-pt 512^3, 8 ranks) at full size, the 8 ranks sharing the box's one
# GPU over the host transport: partition set, per-rank load, V-cycles, iterations to tol.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
df -h /tmp /dev/shm "$HOME" .. > $O/df_512.txt 2>&1
free -g >> $O/df_512.txt 2>&1
timeout -k 10 1100 python -u bench.py --gpus 8 --n 512 --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/bench_g8_512.json 2> $O/bench_g8_512.err || { echo "bench g8 512 failed rc=$?"; tail -30 $O/bench_g8_512.err; exit 1; }
head -c 1500 $O/bench_g8_512.json; echo
