# round 6: circuit stand-in throughput mode with the free-order threshold lowered (SSS_HIP_FREE_MIN)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/circ_free; mkdir -p $O
for fm in ${FMS:-default 1 20 60}; do
  if [ "$fm" = default ]; then unset SSS_HIP_FREE_MIN; else export SSS_HIP_FREE_MIN=$fm; fi
  timeout -k 10 300 python -u bench.py --workload circuit --no-cpu-baseline --parity-converge 0 --parity-cycles 0 \
      --steps 10 --warmup 3 > $O/b_$fm.json 2> $O/b_$fm.err || { tail -5 $O/b_$fm.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; print(sys.argv[2], round(d['value'],1), 'its', c.get('iterations_to_tol'), c.get('final_relres'), c.get('sum_order'))" $O/b_$fm.json $fm
done
