# round 6: column-ELL relaxation with the products formed at the gathers -- the format tests, then
# the kernel-trace per-level split of a short default bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06/xell
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS} -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -20; exit $rc; }
bash tools/gpu/prof.sh > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
head -4 gpurun_out/prof_levels.txt | tail -3; tail -1 gpurun_out/prof_levels.txt; cp gpurun_out/prof_levels.txt $O/
rm -rf gpurun_out/prof_cur
