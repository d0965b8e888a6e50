# multi-workgroup tail: bitwise tests, then the circuit stand-in's V-cycle rate per workgroup count
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tail.py \
    > $O/tail_wg_tests.log 2>&1 || { tail -30 $O/tail_wg_tests.log; exit 1; }
tail -1 $O/tail_wg_tests.log
for wg in 8 16; do
  SSS_HIP_TAIL_WG=$wg timeout -k 10 300 python -u bench.py --workload circuit --steps 200 --warmup 20 --no-cpu-baseline \
      --converge-max 0 > $O/tail_wg_$wg.json 2> $O/tail_wg_$wg.log || { tail -20 $O/tail_wg_$wg.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/tail_wg_$wg.json').read().strip().splitlines()[-1]);print('wg $wg', d['value'], d['ms_per_step'], d['config'].get('single_workgroup_tail_from_level'), d['config'].get('kernel_launches_per_cycle'))"
done
