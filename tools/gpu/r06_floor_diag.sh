# round 6: tail vs partitioned coarse levels, and the single-GPU engine's per-level times (tools/n8_floor.py)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/floor
mkdir -p "$O"
timeout -k 10 600 python -u tools/n8_floor.py --n 400 --ranks 8 --agg ${AGG:-2500,20000} --only-ranks ${RK:-0,5} \
    --out "$O/diag.json" > "$O/diag.out" 2> "$O/diag.err"
rc=$?; tail -8 "$O/diag.err"; exit $rc
