# level-0 lab: x staged in LDS by offset ranges against the gather kernels (7-pt 400^3 relabeled)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 ./tools/l0_lab 400 20 > $O/l0_stage.txt 2>&1 || { cat $O/l0_stage.txt; exit 1; }
cat $O/l0_stage.txt
