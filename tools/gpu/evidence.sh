# Evidence at HEAD on one GPU lease (ROUND, default r04; COMMIT stamped into the PMC file):
#  1. level-0 PMC traffic of both storages -> profiles/${ROUND}_level0_spmv_pmc.json (the bench reads
#     the newest such file for roofline.traffic)
#  2. smoke, then the default bench -> gpurun_out/bench.json
#  3. the kernel-trace profile of a short bench with its per-level split (prof.sh)
#  4. the SQ occupancy / stall pass (pmc_sq.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ROUND=${ROUND:-r04}
mkdir -p gpurun_out
bash tools/gpu/pmc.sh || exit 1
python3 tools/pmc_summarize.py gpurun_out profiles/${ROUND}_level0_spmv_pmc.json "${COMMIT:-unknown}" > /dev/null || exit 1
cp profiles/${ROUND}_level0_spmv_pmc.json gpurun_out/level0_spmv_pmc.json
rm -rf gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke-ok
timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
head -c 400 gpurun_out/bench.json; echo
bash tools/gpu/prof.sh > gpurun_out/prof.out 2>&1 || { tail -20 gpurun_out/prof.out; exit 1; }
tail -16 gpurun_out/prof_levels.txt
bash tools/gpu/pmc_sq.sh > gpurun_out/pmc_sq.out 2>&1 || { tail -20 gpurun_out/pmc_sq.out; exit 1; }
head -20 gpurun_out/kernels_sq_pmc.txt
