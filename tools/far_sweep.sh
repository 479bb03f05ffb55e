# SC_FAR sweep (design tool; GPU box): per variant, compress/uncompress time (kbench) and the
# decoder's FETCH_SIZE (one PMC pass).  Usage: bash tools/far_sweep.sh <tag> lib...
set -u
O=gpurun_out/$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $O
for L in default "$@"; do
  n=$(basename $L .so)
  if [ "$L" = default ]; then unset SNAPPY_MI355X_LIB; else export SNAPPY_MI355X_LIB=$L; fi
  for op in compress_fast uncompress; do
    timeout -k 10 120 python3 tools/kbench.py --op $op --blocks 10000 --reps 20 > $O/k.log 2>&1 || { echo "$n $op failed"; tail $O/k.log; exit 1; }
    echo "$n: $(grep -v amdgpu.ids $O/k.log | tr '\n' ' ')"
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/$n/p1 -o pass -- \
    python3 tools/kbench.py --op uncompress --blocks 10000 --reps 2 > $O/$n.log 2>&1 || { echo "$n pmc failed"; tail -5 $O/$n.log; exit 1; }
  python3 tools/pmc_summary.py $O/$n k_decompress | grep FETCH
done
unset SNAPPY_MI355X_LIB
