# round 6: A/B of two builds (amg_amd/lib = this tree, amg_amd/lib_ab = the alternative): x after 4
# V-cycles bitwise at 256^3 (7-pt and 27-pt), then the kernel-trace per-level profile of each at 400^3
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06/ab_${TAG:-lib}
mkdir -p "$O"
for st in 7 27; do
  timeout -k 10 300 python -u tools/dump_x.py --n ${DUMP_N:-256} --stencil $st --out "$O/x_new_$st.npy" > "$O/dump_new_$st.log" 2>&1 || { tail "$O/dump_new_$st.log"; exit 1; }
  SSS_AMG_LIB=$PWD/amg_amd/lib_ab/libsss_amg.so timeout -k 10 300 python -u tools/dump_x.py --n ${DUMP_N:-256} --stencil $st --out "$O/x_ab_$st.npy" > "$O/dump_ab_$st.log" 2>&1 || { tail "$O/dump_ab_$st.log"; exit 1; }
  python -c "import numpy as np,sys; a=np.load(sys.argv[1]); b=np.load(sys.argv[2]); print('stencil', sys.argv[3], 'bitwise', np.array_equal(a.view(np.uint64), b.view(np.uint64)), 'max|dx|', float(np.max(np.abs(a-b))))" "$O/x_new_$st.npy" "$O/x_ab_$st.npy" $st
done
bash tools/gpu/prof.sh > "$O/prof_new.out" 2>&1 || { tail -20 "$O/prof_new.out"; exit 1; }
cp gpurun_out/prof_levels.txt "$O/levels_new.txt"; cp gpurun_out/prof_bench.json "$O/bench_new.json"
SSS_AMG_LIB=$PWD/amg_amd/lib_ab/libsss_amg.so bash tools/gpu/prof.sh > "$O/prof_ab.out" 2>&1 || { tail -20 "$O/prof_ab.out"; exit 1; }
cp gpurun_out/prof_levels.txt "$O/levels_ab.txt"; cp gpurun_out/prof_bench.json "$O/bench_ab.json"
echo "== new"; cat "$O/levels_new.txt"; echo "== ab"; cat "$O/levels_ab.txt"
python -c "import json,sys; [print(f, json.load(open(f))['ms_per_step']) for f in sys.argv[1:]]" "$O/bench_new.json" "$O/bench_ab.json"
