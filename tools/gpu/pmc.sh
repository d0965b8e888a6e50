set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$c -o run -- python3 tools/pmc_level0.py 400 5 > gpurun_out/pmc_$c.log 2>&1 || exit 1
echo pmc-$c-ok
done
