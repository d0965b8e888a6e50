set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
echo tests-ok
for f in 2 1; do
timeout -k 10 300 python bench.py --no-cpu-baseline --inner 1 --inner-from $f > gpurun_out/b_from$f.json 2> gpurun_out/b_from$f.err || exit 1
echo bench$f-ok
done
