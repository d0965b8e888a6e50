# fused GS-CF engine with sharded ticket counters: GS + parity suites, then the parity-mode trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gs_engines.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/shards_tests.log 2>&1 || { tail -40 $O/shards_tests.log; exit 1; }
tail -2 $O/shards_tests.log
bash tools/gpu/r05_parity_prof.sh
