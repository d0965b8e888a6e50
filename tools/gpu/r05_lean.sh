# lean formats for the exact smoother: whole GPU suite, then parity mirror time vs helper threads
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/lean_suite.log 2>&1 || { tail -30 $O/lean_suite.log; exit 1; }
tail -1 $O/lean_suite.log
for h in 3 5; do
  SSS_HIP_TIMING=1 SSS_LAB_MIRROR_HELPERS=$h timeout -k 10 300 python -u tools/parity_mirror_time.py --n 400 > $O/lean_pm_$h.log 2>&1 || { tail -20 $O/lean_pm_$h.log; exit 1; }
  echo "helpers $h: $(grep 'parity mirror' $O/lean_pm_$h.log)"
done
