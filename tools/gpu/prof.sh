set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG:-x}
export TMPDIR=/tmp
SSS_HIP_GRAPH=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --converge-max 0 ${BENCH_ARGS} > gpurun_out/prof_${TAG:-x}.log 2>&1 || exit 1
echo prof-ok
