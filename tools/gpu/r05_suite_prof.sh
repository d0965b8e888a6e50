# every -m gpu test, then the kernel-trace profile of a short bench with the per-level split and the
# stored-format rates (vcycle_stored)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/gpu_tests.log | head -30; exit $rc; }
bash tools/gpu/prof.sh > gpurun_out/prof.out 2>&1 || { tail -20 gpurun_out/prof.out; exit 1; }
cat gpurun_out/prof_levels.txt
python3 -c "import json; d=json.load(open('gpurun_out/prof_bench.json')); print(d['value'], d['vcycle_stored']['frac'], d['vcycle_stored']['GBps'], d['roofline']['frac'])"
