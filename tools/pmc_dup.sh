# LDS-array and bank-conflict cycles per instruction group of k_compress_sc (design tool; GPU box):
# the plain build and each SC_DUP variant (tools/build_dup.sh), one PMC pass each.
# Usage: bash tools/pmc_dup.sh <tag> lib...   -> gpurun_out/<tag>/<lib>/...
set -u
O=gpurun_out/$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $O
for L in default "$@"; do
  n=$(basename $L .so)
  if [ "$L" = default ]; then unset SNAPPY_MI355X_LIB; else export SNAPPY_MI355X_LIB=$L; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS -d $O/$n/p1 -o pass -- \
    python3 tools/kbench.py --op ${OP:-compress_fast} --blocks 10000 --reps 2 > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  echo "== $n"; head -1 $O/$n.log; python3 tools/pmc_summary.py $O/$n ${KN:-k_compress_sc}
done
