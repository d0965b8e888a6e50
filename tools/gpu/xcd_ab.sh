# A/B of the XCD-contiguous block mapping (SSS_XCD_REMAP build in amg_amd/lib_xcd) on the
# per-level kernel times of the bench workload; dictionary-tile tests first
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gs_engines.py -k "dictionary" -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/td.log 2>&1
rc=$?; tail -2 gpurun_out/td.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/prof.sh || exit 1
cp gpurun_out/prof_levels.txt gpurun_out/prof_levels_base.txt
cp gpurun_out/prof_bench.json gpurun_out/prof_bench_base.json
SSS_AMG_LIB=$GRAFT_REPO_ROOT/amg_amd/lib_xcd/libsss_amg.so bash tools/gpu/prof.sh || exit 1
cp gpurun_out/prof_levels.txt gpurun_out/prof_levels_xcd.txt
