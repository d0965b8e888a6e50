# circuit stand-in: single-workgroup tail threshold (nonzeros of the first tail level)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
for t in 16384 40000 16384 40000; do
  SSS_HIP_TAIL_NNZ=$t timeout -k 10 300 python -u bench.py --workload circuit --steps 300 --warmup 30 --no-cpu-baseline --converge-max 0 > $O/tailnnz_$t.json 2> $O/tailnnz_$t.log || { tail -20 $O/tailnnz_$t.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/tailnnz_$t.json').read().strip().splitlines()[-1]);print('tail_nnz $t', round(d['value'],1), round(d['ms_per_step'],4), d['config'].get('single_workgroup_tail_from_level'))"
done
