# every -m gpu test, then the kernel-trace profile of a short bench with its per-level split
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/gpu/prof.sh > gpurun_out/prof.out 2>&1 || { tail -20 gpurun_out/prof.out; exit 1; }
cat gpurun_out/prof_levels.txt
