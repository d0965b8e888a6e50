# the whole GPU suite at HEAD, then the default bench (N = 1)
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/r05_suite.sh && TAG=head2 bash tools/gpu/r05_bench_default.sh
