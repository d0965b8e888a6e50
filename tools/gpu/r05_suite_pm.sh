# every -m gpu test, the parity mirror's construction phases, then the default bench without CPU baselines
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/gpu_tests.log | head -30; exit $rc; }
SSS_HIP_TIMING=2 timeout -k 10 300 python -u tools/parity_mirror_time.py --n 400 > gpurun_out/parity_mirror_phases.txt 2>&1 || { tail -20 gpurun_out/parity_mirror_phases.txt; exit 1; }
grep "\[pm\]" gpurun_out/parity_mirror_phases.txt
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench.json')); c=d['config']; p=d['parity_mode']
print('value', d['value'], 'iters', c['iterations_to_tol'], c['reference_convergence']['ladder'], 'setup', c['setup_s'], 'upload', c['upload_s'], 'parity', p['value'], 'parity upload', p['upload_s'], 'stored frac', d['vcycle_stored']['frac'], 'roofline', d['roofline']['frac'])"
