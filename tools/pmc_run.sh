#!/bin/bash
# PMC passes for one kernel op (run on the GPU box): tools/pmc_run.sh <op> <outdir> [data]
# Each pass is its own rocprofv3 run (counters only with --kernel-trace, as the pool requires).
set -u
OP=$1; OUT=$2; DATA=${3:-text}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SENDMSG GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $P -d "$OUT/p$i" -o pass -- \
    python3 tools/kbench.py --op "$OP" --blocks ${BLOCKS:-2000} --reps 3 --data "$DATA" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo done
