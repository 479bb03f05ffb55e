# Decoder ablations and stamps (design measurements; GPU box): tools/gpu_dec.sh <tag>
set -u
O=gpurun_out/$1
mkdir -p $O
for L in default tools/abl/lib_d1.so tools/abl/lib_d2.so tools/abl/lib_d4.so; do
  if [ "$L" = default ]; then unset SNAPPY_MI355X_LIB; else export SNAPPY_MI355X_LIB=$L; fi
  timeout -k 10 120 python3 tools/kbench.py --op uncompress --blocks 10000 --reps 20 > $O/k.log 2>&1 || { echo "$L failed"; tail $O/k.log; exit 1; }
  echo "$L: $(grep -v amdgpu.ids $O/k.log | head -1)"
done
export SNAPPY_MI355X_LIB=tools/abl/lib_stamp.so
timeout -k 10 120 python3 tools/stamp_run.py > $O/stamps.log 2>&1 || { echo stamps failed; tail $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log
