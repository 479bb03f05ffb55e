set -u
O=gpurun_out/fine; mkdir -p $O; : > $O/paths.txt
SNAPPY_MI355X_LIB=tools/ablib/lib_fine9.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "small or uncompress or path" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc = 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
for l in fine6 fine9 fine6 fine9; do
  echo "== $l" >> $O/paths.txt
  SNAPPY_MI355X_LIB=tools/ablib/lib_$l.so timeout -k 10 200 python3 tools/single_paths.py >> $O/paths.txt 2>$O/err.txt || { tail $O/err.txt; exit 1; }
done
cat $O/paths.txt | cut -c1-75
