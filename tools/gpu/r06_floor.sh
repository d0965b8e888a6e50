# round 6: the N = 8 per-rank compute floor at 400^3 over replicated-tail thresholds (tools/n8_floor.py)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/floor
mkdir -p "$O"
timeout -k 10 900 python -u tools/n8_floor.py --n ${N:-400} --ranks ${RANKS:-8} --agg ${AGG:-2500,5000,20000,80000,300000} \
    --out "$O/n8_floor_${N:-400}.json" > "$O/n8_floor_${N:-400}.out" 2> "$O/n8_floor_${N:-400}.err"
rc=$?; tail -5 "$O/n8_floor_${N:-400}.err"; exit $rc
