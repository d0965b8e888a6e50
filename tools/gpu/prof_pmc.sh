# kernel-trace profile + per-level breakdown (prof.sh), then the level-0 PMC passes (pmc.sh),
# summarised into gpurun_out/level0_spmv_pmc.json
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/prof.sh || exit 1
bash tools/gpu/pmc.sh || exit 1
python3 tools/pmc_summarize.py gpurun_out gpurun_out/level0_spmv_pmc.json
