# parity tests (bitwise coarse Krylov, exact smoother, block-row chains) + parity-mode kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gs_engines.py tests/test_gpu_pcg.py tests/test_gpu_at_size.py -x -q --timeout 300 --timeout-method thread > $O/krylov_pipe_tests.log 2>&1 || { tail -40 $O/krylov_pipe_tests.log; exit 1; }
tail -3 $O/krylov_pipe_tests.log
bash tools/gpu/r05_parity_prof.sh
