# A/B timing of library variants (design tool; run on the GPU box): tools/gpu_ab.sh <tag> lib...
# the in-tree library first, then each variant, twice in alternation; kbench checks the round trip
set -u
O=gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  for L in default "$@"; do
    if [ "$L" = default ]; then unset SNAPPY_MI355X_LIB; else export SNAPPY_MI355X_LIB=$L; fi
    timeout -k 10 120 python3 tools/kbench.py --op ${OP:-compress_fast} --blocks 10000 --reps 20 > $O/k.log 2>&1 || { echo "$L failed"; tail $O/k.log; exit 1; }
    echo "$L: $(grep -v amdgpu.ids $O/k.log | tr '\n' ' ')"
  done
done
unset SNAPPY_MI355X_LIB
