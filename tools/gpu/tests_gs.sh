# every -m gpu test, the per-level exact GS-CF times at 256^3 (flow engine), the throughput profile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u tools/gs_level_times.py --n 256 --engines flow --reps 3 --json gpurun_out/gs_levels.json > gpurun_out/gs_levels.txt 2>&1 || { tail -20 gpurun_out/gs_levels.txt; exit 1; }
grep "^\[gs\] flow" gpurun_out/gs_levels.txt
bash tools/gpu/prof.sh > gpurun_out/prof.out 2>&1 || { tail -20 gpurun_out/prof.out; exit 1; }
cat gpurun_out/prof_levels.txt
