# Partition sets of the multi-GPU BASELINE configs, built on the GPU box's host (no GPU use):
# by default 27-pt anisotropic 256^3 over 4 ranks and 7-pt 512^3 over 8 ranks ($CFGS: others).  Each manifest records the
# setup and partition seconds, the partitioning process's peak RSS, per-rank file sizes, ghosts
# and peers per level (amg_amd/partition.py).  The partition files themselves stay on the box.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/parts
df -h /tmp > gpurun_out/parts/df.txt 2>&1
free -g >> gpurun_out/parts/df.txt 2>&1
D=${SSS_PART_DIR:-/tmp}
CFGS=${CFGS:-"27,256,4 7,512,8"}   # stencil,n,ranks triples
for cfg in $CFGS; do
    set -- ${cfg//,/ }
    pre="$D/sss_parts_${1}pt_${2}_${3}r/part"
    echo "== ${1}-pt ${2}^3 over ${3} ranks -> $pre" >&2
    timeout -k 10 900 python -u -m amg_amd.partition --stencil "$1" --n "$2" --ranks "$3" --prefix "$pre" \
        > "gpurun_out/parts/p${1}_${2}_${3}.out" 2> "gpurun_out/parts/p${1}_${2}_${3}.err" || { tail -20 "gpurun_out/parts/p${1}_${2}_${3}.err"; exit 1; }
    cp "$pre.json" "gpurun_out/parts/p${1}_${2}_${3}.json"
    ls -l "$(dirname "$pre")" >> gpurun_out/parts/df.txt
    cat "gpurun_out/parts/p${1}_${2}_${3}.out"
    rm -rf "$(dirname "$pre")"
done
df -h /tmp >> gpurun_out/parts/df.txt 2>&1
