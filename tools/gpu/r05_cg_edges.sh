# coarse Krylov tests (register CG step size edges) + smoke()
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "coarse_krylov" -x -q --timeout 200 --timeout-method thread > $O/cg_edges.log 2>&1 || { tail -30 $O/cg_edges.log; exit 1; }
tail -2 $O/cg_edges.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
