set -u
O=gpurun_out/tb; mkdir -p $O; : > $O/paths.txt
SNAPPY_MI355X_LIB=tools/ablib/lib_tb65536.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc = 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
for l in tb16384 tb32768 tb65536 tb16384 tb32768 tb65536; do
  echo "== $l" >> $O/paths.txt
  SNAPPY_MI355X_LIB=tools/ablib/lib_$l.so timeout -k 10 200 python3 tools/single_paths.py >> $O/paths.txt 2>$O/err.txt || { tail $O/err.txt; exit 1; }
done
cat $O/paths.txt | cut -c1-75
