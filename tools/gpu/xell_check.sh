# column ELL: the storage-format and per-level SpMV parity tests, then an A/B of the per-level
# kernel times at the bench workload (column ELL off / on)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gs_engines.py tests/test_gpu_parity.py -k "dictionary_tiles or spmv or parity_solve" -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/xell_tests.log 2>&1 || { tail -40 gpurun_out/xell_tests.log; exit 1; }
tail -3 gpurun_out/xell_tests.log
bash tools/gpu/ab.sh noxell=SSS_HIP_XELL=0 xell=SSS_HIP_XELL=1
