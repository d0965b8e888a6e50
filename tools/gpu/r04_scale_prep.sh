# The 400^3 partition sets of bench.py --gpus 2/4/8 (built on the box's host, no GPU), then the
# default 1-GPU bench at HEAD
cd "$GRAFT_REPO_ROOT" || exit 1
CFGS="7,400,2 7,400,4 7,400,8" bash tools/gpu/partitions.sh || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
head -c 600 gpurun_out/bench.json; echo
