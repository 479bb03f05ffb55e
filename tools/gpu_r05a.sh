# Round-5 decoder/compressor measurement batch (design tool, GPU box): GPU suite, same-box A/B of
# the product against HEAD~ builds and variants, section PMC of the duplication builds, stamps.
set -u
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { echo "pytest rc $rc"; exit 1; }
timeout -k 10 300 python tools/ab_raw.py --rounds 3 tools/ablib/lib_head.so snappy.jl_amd/libsnappy_mi355x.so \
  tools/ablib/lib_queue.so tools/ablib/lib_cet.so tools/ablib/lib_far0.so tools/ablib/lib_far128.so tools/ablib/lib_far512.so > $O/ab.log 2>&1 \
  || { echo "ab rc $?"; tail -5 $O/ab.log; exit 1; }
grep -v "^round" $O/ab.log
ABFLAGS=--decode-ablation bash tools/pmc_quick.sh $O/pmc snappy.jl_amd/libsnappy_mi355x.so tools/ablib/lib_dup1.so \
  tools/ablib/lib_dup2.so tools/ablib/lib_dup4.so tools/ablib/lib_dup8.so || exit 1
SNAPPY_MI355X_LIB=tools/ablib/lib_stamp_new.so timeout -k 10 120 python3 tools/stamp_run.py > $O/stamps.log 2>&1 || { echo stamps failed; exit 1; }
grep -v amdgpu.ids $O/stamps.log
