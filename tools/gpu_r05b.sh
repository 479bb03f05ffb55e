# Round-5 compressor section costs (design tool, GPU box): timing and instruction counts of the
# SC_ABL ablation builds (invalid output: timing only) against the product; single-call A/B r04 vs now.
set -u
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python tools/ab_raw.py --rounds 3 --no-verify --compress-only snappy.jl_amd/libsnappy_mi355x.so \
  tools/ablib/lib_sabl1.so tools/ablib/lib_sabl2.so tools/ablib/lib_sabl16.so tools/ablib/lib_sabl32.so > $O/ab.log 2>&1 \
  || { echo "ab rc $?"; tail -5 $O/ab.log; exit 1; }
grep -v "^round" $O/ab.log
ABFLAGS="--no-verify --compress-only" bash tools/pmc_quick.sh $O/pmc snappy.jl_amd/libsnappy_mi355x.so tools/ablib/lib_sabl1.so tools/ablib/lib_sabl2.so \
  tools/ablib/lib_sabl16.so tools/ablib/lib_sabl32.so || exit 1
bash tools/single_call_ab.sh tools/ablib/lib_r04.so snappy.jl_amd/libsnappy_mi355x.so
