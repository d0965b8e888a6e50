# parity mirror phases at 400^3
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
SSS_HIP_TIMING=2 timeout -k 10 400 python -u tools/parity_mirror_time.py --n 400 > $O/pm_phases.log 2>&1 || { tail -20 $O/pm_phases.log; exit 1; }
grep -E "\[pm\]" $O/pm_phases.log
