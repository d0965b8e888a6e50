# round 6: the one-launch coarse CG -- the coarse-solve and parity-solve GPU tests, then the parity
# cycle at 400^3 with it and with two kernels per iteration (SSS_HIP_CG_PERSIST=0)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/cg
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "coarse_krylov or solve_parity or bus_known or drop_in or hybrid_krylov or reference_main" > "$O/tests.log" 2>&1
rc=$?; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" "$O/tests.log" | head -30; exit $rc; }
[ -n "$NO_BENCH" ] && exit 0
for v in 1 0; do
  SSS_HIP_CG_PERSIST=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --parity-cycles 3 --parity-converge 0 \
      --converge-max 0 --steps 2 --warmup 1 > "$O/bench_persist$v.json" 2> "$O/bench_persist$v.err"
  rc=$?; [ $rc -eq 0 ] || { tail -20 "$O/bench_persist$v.err"; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['parity_mode']; print('persist', sys.argv[2], 'parity ms/cycle', p['ms_per_step'], 'relres', p['relres_first_cycles'])" "$O/bench_persist$v.json" $v
done
