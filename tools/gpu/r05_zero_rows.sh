# fused engine: sweep-0 rows without the zero-iterate entries -- GS and parity tests, then the default bench
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_engines.py tests/test_gpu_parity.py > $O/zr_tests.log 2>&1 || { tail -30 $O/zr_tests.log; exit 1; }
tail -1 $O/zr_tests.log
TAG=zero_rows bash tools/gpu/r05_bench_default.sh
