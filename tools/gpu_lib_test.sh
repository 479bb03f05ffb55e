# GPU suite + A/B timing for a candidate library (GPU box): tools/gpu_lib_test.sh <tag> <lib> <op>
set -u
O=gpurun_out/$1; L=$2; OP=${3:-uncompress}
mkdir -p $O
SNAPPY_MI355X_LIB=$L timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc = 0 ] || { echo "pytest rc $rc"; exit 1; }
for rep in 1 2; do
  for X in default $L; do
    if [ "$X" = default ]; then unset SNAPPY_MI355X_LIB; else export SNAPPY_MI355X_LIB=$X; fi
    timeout -k 10 120 python3 tools/kbench.py --op $OP --blocks 10000 --reps 20 > $O/k.log 2>&1 || { echo "$X failed"; tail $O/k.log; exit 1; }
    echo "$X: $(grep -v amdgpu.ids $O/k.log | tr '\n' ' ')"
  done
done
