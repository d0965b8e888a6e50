# throughput-mode smoother variants to tol at 7-pt 512^3 (reference semantics: 73 iterations, measured
# by the parity mirror in gpurun_out/r05/bench_n1_512.json): which one keeps the ref + 2 ladder
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 1100 python -u tools/conv_study.py --n 512 --maxit 90 --modes throughput,hyb:1:1,hyb:2:2,hyb:2:1 \
    --json $O/conv512.json > $O/conv512.log 2>&1 || { tail -20 $O/conv512.log; exit 1; }
grep "iterations, upload" $O/conv512.log
