set -u
O=gpurun_out/spin; mkdir -p $O; : > $O/paths.txt
for l in spin0 spin1 spin0 spin1; do
  echo "== $l" >> $O/paths.txt
  SNAPPY_MI355X_LIB=tools/ablib/lib_$l.so timeout -k 10 200 python3 tools/single_paths.py >> $O/paths.txt 2>$O/err.txt || { tail $O/err.txt; exit 1; }
done
cat $O/paths.txt
