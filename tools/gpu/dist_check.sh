# every -m gpu test, then bench.py --gpus 2 on the one GPU (two ranks, host transport fallback)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/gpu_tests.log | head -30; exit $rc; }
SSS_PART_DIR=$GRAFT_REPO_ROOT/gpurun_out/parts timeout -k 10 600 python -u bench.py --gpus 2 --n 64 --steps 5 --warmup 2 > gpurun_out/bench2.json 2> gpurun_out/bench2.err
rc=$?; cat gpurun_out/bench2.json; tail -5 gpurun_out/bench2.err; rm -rf gpurun_out/parts; exit $rc
