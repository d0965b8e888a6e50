# 400^3: upload phase times, throughput vs parity (reference semantics) histories and V-cycle times
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SSS_HIP_TIMING=1 timeout -k 10 1000 python -u tools/conv_study.py --n ${N:-400} --modes ${MODES:-throughput,parity} --maxit ${MAXIT:-45} --json gpurun_out/conv${N:-400}.json > gpurun_out/conv${N:-400}.log 2>&1
rc=$?; grep "\[conv\].*iterations" gpurun_out/conv${N:-400}.log; exit $rc
