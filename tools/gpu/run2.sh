set -o pipefail
cd $GRAFT_REPO_ROOT
for m in 2 1; do
SSS_HIP_RELABEL=$m timeout -k 10 300 python bench.py --no-cpu-baseline --converge-max 0 > gpurun_out/b_relabel$m.json 2> gpurun_out/b_relabel$m.err || exit 1
echo bench$m-ok
done
