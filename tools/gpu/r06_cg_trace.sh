# round 6: phase timestamps of the one-launch coarse CG (SSS_HIP_CG_TRACE=1, first launch) in the
# parity mode at 400^3, after the coarse-solve GPU tests
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/cg_trace
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "coarse_krylov" > "$O/tests.log" 2>&1
rc=$?; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" "$O/tests.log" | head -30; exit $rc; }
SSS_HIP_CG_TRACE=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --parity-cycles 3 --parity-converge 0 \
    --converge-max 0 --steps 2 --warmup 1 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; grep "cg trace" "$O/bench.err"; [ $rc -eq 0 ] || { tail -20 "$O/bench.err"; exit $rc; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['parity_mode']; print('parity ms/cycle', p['ms_per_step'])" "$O/bench.json"
