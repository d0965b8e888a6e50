# time to solution of smoother variants at the bench workload (hierarchy set up once, cached in /tmp)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/study
common="--no-cpu-baseline --parity-cycles 0 --parity-converge 0 --steps 5 --warmup 2 --hier-cache /tmp/h400.bin"
for v in "base:" "if1:--inner-from 1" "in2:--inner 2" "in2if1:--inner 2 --inner-from 1" "in0:--inner 0"; do
    label=${v%%:*}; args=${v#*:}
    timeout -k 10 400 python -u bench.py $common $args > gpurun_out/study/$label.json 2> gpurun_out/study/$label.err || { echo "$label failed"; tail -5 gpurun_out/study/$label.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/study/$label.json')); c=d['config']
print('$label', round(d['value'],2), 'cyc/s', round(d['ms_per_step'],3), 'ms', 'iters', c['iterations_to_tol'], 'tts', round(c['time_to_solution_s'],4), 'pcg', c['amg_pcg']['iterations_to_tol'], round(c['amg_pcg']['time_to_solution_s'],4))"
done
