# upload A/B: single-call times per build (pageable H2D / pinned staging + DMA / + copy kernel)
set -u
O=gpurun_out/up; mkdir -p $O
for l in up0 up1 up2 up0 up1 up2; do
  echo "== $l" >> $O/paths.txt
  SNAPPY_MI355X_LIB=tools/ablib/lib_$l.so timeout -k 10 200 python3 tools/single_paths.py >> $O/paths.txt 2>$O/err_$l.txt || { echo paths $l failed; tail $O/err_$l.txt; exit 1; }
done
SNAPPY_MI355X_LIB=tools/ablib/lib_up2.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "single or pinned or small or validate" > $O/pytest_up2.log 2>&1 || { echo pytest failed; tail -30 $O/pytest_up2.log; exit 1; }
tail -2 $O/pytest_up2.log; cat $O/paths.txt
