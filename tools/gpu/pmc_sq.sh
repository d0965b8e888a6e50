# occupancy and stall counters per kernel shape over a short 400^3 bench (one --pmc pass, SQ + GRBM)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_sq
SSS_HIP_GRAPH=0 timeout -s KILL 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_sq -o run -- python3 bench.py --steps 2 --warmup 1 --converge-max 0 --parity-cycles 0 --parity-converge 0 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/pmc_sq.log 2>&1 || { tail -20 gpurun_out/pmc_sq.log; exit 1; }
python3 tools/pmc_kernels.py gpurun_out/pmc_sq 60 > gpurun_out/kernels_sq_pmc.txt
head -45 gpurun_out/kernels_sq_pmc.txt
rm -rf gpurun_out/pmc_sq
