# 27-pt anisotropic: the 64^3 GPU tests, then 256^3 at full size on one GPU -- the throughput bench
# with the parity mirror run to tol in the same process (hybrid smoother), and the 4-rank
# configuration's smoother (C/F-Jacobi on level 0) for its iteration count
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_a27.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/a27_tests.log 2>&1
rc=$?; tail -3 gpurun_out/a27_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/a27_tests.log | head -30; exit $rc; }
SSS_SETUP_TIMING=1 SSS_HIP_TIMING=1 timeout -k 10 900 python -u bench.py --stencil 27 --n 256 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_a27.json 2> gpurun_out/bench_a27.err || { tail -30 gpurun_out/bench_a27.err; exit 1; }
head -c 400 gpurun_out/bench_a27.json; echo
timeout -k 10 600 python -u bench.py --stencil 27 --n 256 --no-cpu-baseline --mode-smoother jacobi --parity-cycles 0 --steps 10 --warmup 3 > gpurun_out/bench_a27_jacobi.json 2> gpurun_out/bench_a27_jacobi.err || { tail -30 gpurun_out/bench_a27_jacobi.err; exit 1; }
head -c 400 gpurun_out/bench_a27_jacobi.json; echo
