# the bench's N > 1 path on one GPU (ranks share the device; RCCL refuses that, so all ranks take
# the host transport together): N = 2 (7-pt), N = 4 (27-pt, level 0 by C/F-Jacobi), N = 8 (7-pt)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "2:--n 64" "4:--stencil 27 --n 48" "8:--n 64"; do
    N=${v%%:*}; args=${v#*:}
    timeout -k 10 400 python -u bench.py --gpus $N $args --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_g$N.json 2> gpurun_out/bench_g$N.err || { echo "N=$N failed"; tail -20 gpurun_out/bench_g$N.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/bench_g$N.json')); c=d['config']
print('N=$N', round(d['value'],2), d['unit'], round(d['ms_per_step'],3), 'ms', c['workload'], 'transport', c.get('transport'), 'iters', c.get('iterations_to_tol'), 'parallelism', c.get('parallelism'))"
done
