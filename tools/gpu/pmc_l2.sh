# L2 hit/miss and L1->L2 read requests per kernel shape over a short bench run (one --pmc pass)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_l2
SSS_HIP_GRAPH=0 timeout -s KILL 500 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_l2 -o run -- python3 bench.py --steps 2 --warmup 1 --converge-max 0 --parity-cycles 0 --no-cpu-baseline > gpurun_out/pmc_l2.log 2>&1 || { tail -20 gpurun_out/pmc_l2.log; exit 1; }
python3 tools/pmc_levels.py gpurun_out/pmc_l2 > gpurun_out/levels_l2_pmc.txt
cat gpurun_out/levels_l2_pmc.txt
rm -rf gpurun_out/pmc_l2
