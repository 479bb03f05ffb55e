# VALU/SALU/LDS instruction counts per library variant (design tool; GPU box): tools/pmc_abl.sh <tag> lib...
set -u
O=gpurun_out/$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $O
for L in default "$@"; do
  n=$(basename $L .so)
  if [ "$L" = default ]; then unset SNAPPY_MI355X_LIB; else export SNAPPY_MI355X_LIB=$L; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $O/$n/p1 -o pass -- \
    python3 tools/kbench.py --op ${OP:-compress_fast} --blocks 10000 --reps 2 > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  echo "== $n"; python3 tools/pmc_summary.py $O/$n ${KN:-k_compress_sc}
done
