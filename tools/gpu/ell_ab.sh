# ELL kernels: one-shot blocks in dispatch order vs XCD-contiguous order (SSS_HIP_ELL_REMAP),
# per-level profile of each, and the level-0 SpMV HBM traffic of each
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rm in 0 1; do
  SSS_HIP_ELL_REMAP=$rm bash tools/gpu/prof.sh > gpurun_out/prof_ell_$rm.txt 2>&1 || { tail gpurun_out/prof_ell_$rm.txt; exit 1; }
  grep -E "^    [01] |^total|^   out" gpurun_out/prof_ell_$rm.txt
  for c in FETCH_SIZE WRITE_SIZE; do
    SSS_HIP_ELL_REMAP=$rm timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$c -o run -- python3 tools/pmc_level0.py 400 5 > gpurun_out/pmc_$c.log 2>&1 || exit 1
  done
  python3 tools/pmc_summarize.py gpurun_out gpurun_out/level0_spmv_pmc_remap$rm.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('remap', $rm, 'ms', d['avg_ms_under_pmc_pass'], 'hbm GB', d['hbm_bytes_per_launch']/1e9, 'alg GB', d['algorithmic_bytes_per_launch']/1e9)"
  rm -rf gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE
done
