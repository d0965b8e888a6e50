# round 6 evidence, lease 1: level-0 PMC traffic (profiles/r06_level0_spmv_pmc.json, read by the bench
# for roofline.traffic), then smoke() and the default bench line in the same lease
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/evidence
bash tools/gpu/pmc.sh || exit 1
python3 tools/pmc_summarize.py gpurun_out profiles/r06_level0_spmv_pmc.json "${COMMIT:-unknown}" > /dev/null || exit 1
cp profiles/r06_level0_spmv_pmc.json gpurun_out/r06/evidence/level0_spmv_pmc.json
rm -rf gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/evidence/smoke.log 2>&1 || { tail -20 gpurun_out/r06/evidence/smoke.log; exit 1; }
echo smoke-ok
timeout -k 10 900 python -u bench.py > gpurun_out/r06/evidence/bench.json 2> gpurun_out/r06/evidence/bench.err || { tail -20 gpurun_out/r06/evidence/bench.err; exit 1; }
head -c 600 gpurun_out/r06/evidence/bench.json; echo
