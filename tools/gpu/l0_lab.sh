# level-0 rows-per-thread lab (tools/l0_lab.hip, prebuilt in-tree), then the distributed GPU tests
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 ./tools/l0_lab 400 20 > gpurun_out/l0_lab.txt 2>&1 || { cat gpurun_out/l0_lab.txt; exit 1; }
cat gpurun_out/l0_lab.txt
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dist_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/dist_gpu.log; exit $rc
