# the default bench (as the driver runs it), then the SQ occupancy/stall pass
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
head -c 300 gpurun_out/bench.json; echo
bash tools/gpu/pmc_sq.sh
