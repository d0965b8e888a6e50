# W-cycle in throughput mode against the oracle (before / after the zero-iterate fix)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "w_cycle" > $O/wcycle.log 2>&1
rc=$?; tail -15 $O/wcycle.log; exit $rc
