# round 6: kernel trace of the parity mode at 400^3 (coarse CG one launch vs two kernels per iteration)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06/cg_prof
mkdir -p "$O"
for v in ${VARIANTS:-1 0}; do
  rm -rf "$O/p$v"
  SSS_HIP_CG_PERSIST=$v timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/p$v" -o run --output-format csv -- \
      python3 bench.py --mode parity --steps 2 --warmup 1 --no-cpu-baseline --converge-max 0 --parity-cycles 0 \
      > "$O/p$v.log" 2>&1 || { tail -20 "$O/p$v.log"; exit 1; }
  f=$(find "$O/p$v" -name '*kernel_stats.csv' | head -1)
  echo "== persist $v"; head -14 "$f" | cut -d, -f1-5 | cut -c1-160
done
