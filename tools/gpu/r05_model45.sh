# lanes-per-row model with the sharded tickets' 4.5 ns: 400^3 parity trace, then the irregular workloads
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/r05_parity_prof.sh && bash tools/gpu/r05_irregular_parity.sh
