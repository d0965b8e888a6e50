# host setup at 400^3 with and without transparent huge pages on the large host arrays
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > $O/thp_settings.txt 2>&1
for mode in huge nohuge huge; do
  if [ $mode = nohuge ]; then export SSS_NO_HUGEPAGE=1; else unset SSS_NO_HUGEPAGE; fi
  SSS_SETUP_TIMING=1 timeout -k 10 200 python -u tools/setup_time.py --n 400 > $O/setup_$mode.log 2>&1 || { tail -5 $O/setup_$mode.log; exit 1; }
  echo "== $mode"; grep -E "first pass|setup_time|level [0-2]:" $O/setup_$mode.log | head -8
done
cat $O/thp_settings.txt
