#!/bin/bash
# PMC comparison of library variants on one op: tools/pmc_ab.sh <op> <data> <outdir> lib1.so lib2.so ...
set -u
OP=$1; DATA=$2; OUT=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in "$@"; do
  tag=$(basename $L .so)
  mkdir -p "$OUT/$tag"
  i=0
  for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SENDMSG GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM"; do
    i=$((i+1))
    SNAPPY_MI355X_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $P -d "$OUT/$tag/p$i" -o pass -- \
      python3 tools/kbench.py --op "$OP" --blocks ${BLOCKS:-4000} --reps 2 --data "$DATA" > "$OUT/$tag/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/$tag/p$i.log"; exit 1; }
  done
  python3 tools/pmc_summary.py $OUT/$tag ${KF:-k_compress} > $OUT/$tag.txt
done
echo done
