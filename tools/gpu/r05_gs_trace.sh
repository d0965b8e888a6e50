# exact GS-CF flow engine: critical-path statistics of levels 3-9 at 7-pt 400^3 (diagnostic trace build)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f /tmp/gs_trace.bin
SSS_AMG_LIB=$GRAFT_REPO_ROOT/amg_amd/lib_trace/libsss_amg.so SSS_GS_TRACE_FILE=/tmp/gs_trace.bin timeout -k 10 400 \
    python -u tools/gs_level_times.py --n 400 --engines flow --levels 3,4,5,6,7,8,9 --reps 1 > gpurun_out/gs_trace_levels.txt 2>&1 || { tail -20 gpurun_out/gs_trace_levels.txt; exit 1; }
grep "\[gs\]" gpurun_out/gs_trace_levels.txt
python3 tools/gs_trace_stats.py /tmp/gs_trace.bin > gpurun_out/gs_trace_stats.txt 2>&1; cat gpurun_out/gs_trace_stats.txt
SSS_HIP_TIMING=2 timeout -k 10 300 python -u tools/parity_mirror_time.py --n 400 > gpurun_out/parity_mirror_phases.txt 2>&1 || { tail -20 gpurun_out/parity_mirror_phases.txt; exit 1; }
grep -v "cpu_step" gpurun_out/parity_mirror_phases.txt | grep "sss_hip\|\[pm\]" | tail -60
