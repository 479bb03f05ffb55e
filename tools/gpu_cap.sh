# rewalk-cap A/B: timing on text + large, per-file sizes per build
set -u
O=gpurun_out/cap; mkdir -p $O
timeout -k 10 300 python3 tools/ab_raw.py --rounds 3 tools/ablib/lib_base.so tools/ablib/lib_cap2.so tools/ablib/lib_cap3.so > $O/text.log 2>&1 || { tail -20 $O/text.log; exit 1; }
timeout -k 10 300 python3 tools/ab_raw.py --rounds 3 --data large tools/ablib/lib_base.so tools/ablib/lib_cap2.so tools/ablib/lib_cap3.so > $O/large.log 2>&1 || { tail -20 $O/large.log; exit 1; }
for l in base cap2 cap3; do
  SNAPPY_MI355X_LIB=tools/ablib/lib_$l.so timeout -k 10 200 python3 -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "test_fast_mode_sizes_per_corpus_file" > $O/sizes_$l.log 2>&1 || { echo sizes $l failed; tail -30 $O/sizes_$l.log; }
done
grep -v amdgpu.ids $O/text.log | tail -4; grep -v amdgpu.ids $O/large.log | tail -4; grep -h "worst\|passed\|failed" $O/sizes_*.log
