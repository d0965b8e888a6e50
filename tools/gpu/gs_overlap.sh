# exact GS-CF engines: the bitwise GS tests, then per-level pre-smoother times at 256^3 with the
# flow engine's chain/poll overlap off and on (SSS_HIP_GS_OVERLAP)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_gs_engines.py tests/test_gpu_parity.py tests/test_gpu_circuit.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gs_tests.log 2>&1 || { tail -30 gpurun_out/gs_tests.log; exit 1; }
tail -2 gpurun_out/gs_tests.log
for o in 0 1; do
  SSS_HIP_GS_OVERLAP=$o timeout -k 10 300 python -u tools/gs_level_times.py --n ${N:-256} --engines flow --reps 3 --json gpurun_out/gs_levels_ovl$o.json > gpurun_out/gs_levels_ovl$o.txt 2>&1 || { tail -20 gpurun_out/gs_levels_ovl$o.txt; exit 1; }
  echo "== overlap $o"; cat gpurun_out/gs_levels_ovl$o.txt
done
