set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; exit 1; }
echo tests-ok
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_relabel.json 2> gpurun_out/b_relabel.err || exit 1
echo bench1-ok
SSS_HIP_RELABEL=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_norelabel.json 2> gpurun_out/b_norelabel.err || exit 1
echo bench2-ok
