# host-side phase timings at the bench workload: setup (SSS_SETUP_TIMING) and upload (SSS_HIP_TIMING)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SSS_SETUP_TIMING=1 SSS_HIP_TIMING=${HIPT:-1} timeout -k 10 900 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
  --converge-max 0 --parity-cycles 0 ${BENCH_ARGS} > gpurun_out/phases.json 2> gpurun_out/phases.err
rc=$?; grep -v "^ \|^---" gpurun_out/phases.err | tail -60; cat gpurun_out/phases.json | head -c 600; exit $rc
