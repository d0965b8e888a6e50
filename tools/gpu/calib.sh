set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/calib -o run -- tools/pmc_calib > gpurun_out/calib.log 2>&1 || exit 1
echo calib-ok
