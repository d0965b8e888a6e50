# run-coded dictionary ELL: bitwise on/off tests, the parity suite, then an A/B of the per-level
# kernel times at the bench workload (runs on / off)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ell_runs.py tests/test_gpu_parity.py tests/test_gpu_ledger.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/runs_tests.log 2>&1 || { tail -40 gpurun_out/runs_tests.log; exit 1; }
tail -2 gpurun_out/runs_tests.log
bash tools/gpu/ab.sh runs= noruns=SSS_HIP_ELL_RUNS=0 || exit 1
for v in runs noruns; do head -3 gpurun_out/ab/levels_$v.txt; done
