# Compress and uncompress A/B of library variants (design tool; GPU box): tools/gpu_ab2.sh <tag> lib...
set -u
O=gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  for L in default "$@"; do
    if [ "$L" = default ]; then unset SNAPPY_MI355X_LIB; else export SNAPPY_MI355X_LIB=$L; fi
    for op in ${OPS:-compress_fast uncompress}; do
      timeout -k 10 120 python3 tools/kbench.py --op $op --blocks 10000 --reps 20 > $O/k.log 2>&1 || { echo "$L $op failed"; tail $O/k.log; exit 1; }
      echo "$L: $(grep -v amdgpu.ids $O/k.log | tr '\n' ' ')"
    done
  done
done
unset SNAPPY_MI355X_LIB
