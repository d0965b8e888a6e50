# merged row groups: 8 vs 4 loads in flight per lane (amg_amd/lib_xcd built with -DSSS_MERGE_U=4)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu/prof.sh > gpurun_out/prof_u8.txt 2>&1 || { tail gpurun_out/prof_u8.txt; exit 1; }
SSS_AMG_LIB=$GRAFT_REPO_ROOT/amg_amd/lib_xcd/libsss_amg.so bash tools/gpu/prof.sh > gpurun_out/prof_u4.txt 2>&1 || exit 1
cat gpurun_out/prof_u8.txt gpurun_out/prof_u4.txt | grep -v "^\[" 
