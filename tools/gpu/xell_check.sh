# column ELL: parity tests of the storage formats, whole solves and the distributed engine, then an
# A/B of the per-level kernel times at the bench workload (${AB:-column ELL on the two-stage copies off / on})
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gs_engines.py tests/test_gpu_parity.py tests/test_dist_gpu.py \
  tests/test_gpu_a27.py tests/test_gpu_circuit.py -x -v --timeout 300 --timeout-method thread > gpurun_out/xell_tests.log 2>&1 || { tail -40 gpurun_out/xell_tests.log; exit 1; }
tail -3 gpurun_out/xell_tests.log
bash tools/gpu/ab.sh ${AB:-noxellts=SSS_HIP_XELL_TS=0 xell=SSS_HIP_XELL_TS=1}
