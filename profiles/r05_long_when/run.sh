# lab: where the long-row levels' extra inner step applies (all passes / post-smoother / pre / F / C)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05; mkdir -p $O
N=${N:-512}
timeout -k 10 1100 python -u tools/conv_study.py --n $N --maxit 90 --modes throughput,w:post,w:pre,w:F,w:C \
    --json $O/long_when_$N.json > $O/long_when_$N.log 2>&1 || { tail -20 $O/long_when_$N.log; exit 1; }
grep "iterations, upload" $O/long_when_$N.log | cut -d, -f1-3
