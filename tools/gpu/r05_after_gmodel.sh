# after the lanes-per-row model: the whole GPU suite, then the circuit and 27-pt bench lines
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gm_suite.log 2>&1 || { tail -30 $O/gm_suite.log; exit 1; }
tail -1 $O/gm_suite.log
bash tools/gpu/r05_irregular_parity.sh
