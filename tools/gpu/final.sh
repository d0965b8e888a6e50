# Round-end evidence on one GPU: level-0 PMC (CSR arrays and the cycle's storage) into profiles/,
# smoke, then the default bench (it reads the PMC file for roofline.traffic), then the kernel-trace
# profile of the same command with its per-level split.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/pmc.sh || exit 1
python3 tools/pmc_summarize.py gpurun_out profiles/r02_level0_spmv_pmc.json > /dev/null || exit 1
cp profiles/r02_level0_spmv_pmc.json gpurun_out/level0_spmv_pmc.json
rm -rf gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.err; exit $rc; }
bash tools/gpu/prof.sh
# N = 2 on the one-GPU box: two ranks (host transport when RCCL cannot pair two ranks on one GPU)
timeout -k 10 300 python -u bench.py --gpus 2 --n 64 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err
rc=$?; tail -c 400 gpurun_out/bench_g2.json; exit $rc
