# Round 5: BASELINE.json's multi-GPU configs at full size, as ranks sharing the box's one GPU (host
# transport): the 27-pt 256^3 / 4-rank bitwise test, then bench.py --gpus 8 at the metric's 400^3.
# (512^3 / 8 ranks: tools/gpu/r05_dist_512.sh, its own call.)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_dist_at_size.py -x -v -s --timeout 400 --timeout-method thread \
    > $O/t_dist_a27.log 2>&1 || { echo "dist test failed rc=$?"; tail -40 $O/t_dist_a27.log; exit 1; }
tail -3 $O/t_dist_a27.log
timeout -k 10 600 python -u bench.py --gpus 8 --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/bench_g8_400.json 2> $O/bench_g8_400.err || { echo "bench g8 400 failed rc=$?"; tail -30 $O/bench_g8_400.err; exit 1; }
head -c 1500 $O/bench_g8_400.json; echo
