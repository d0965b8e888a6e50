# the whole GPU suite at HEAD (one process), as the driver runs it
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite_head.log 2>&1
rc=$?; tail -5 $O/suite_head.log; exit $rc
