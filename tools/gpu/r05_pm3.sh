# lab: parity mirror wall time vs helper threads
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
for h in 3 5 7 3; do
  SSS_LAB_MIRROR_HELPERS=$h timeout -k 10 300 python -u tools/parity_mirror_time.py --n 400 > $O/pm3_$h.log 2>&1 || { tail -20 $O/pm3_$h.log; exit 1; }
  echo "helpers $h: $(grep 'parity mirror' $O/pm3_$h.log)"
done
