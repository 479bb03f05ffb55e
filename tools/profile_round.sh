#!/bin/bash
# One round's profiles (run on the GPU box): tools/profile_round.sh <round>   e.g. r02
# 1. rocprofv3 kernel trace + stats of the bench command (bench.py --no-cpu);
# 2. per-workload kernel traces of tools/kbench.py (text / random, compress / uncompress);
# 3. PMC passes (tools/pmc_run.sh) of the text and random compress/uncompress kernels, 10K blocks.
# Writes gpurun_out/<round>_prof/...; tools/pmc_json.py then makes profiles/<round>_pmc.json.
set -u
R=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${R}_prof
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
  python3 bench.py --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench trace failed"; tail -5 "$OUT/bench.err"; exit 1; }
# per-workload kernel traces (one op, one workload per run, so each kernel's average is that
# workload's launch duration -- the bench trace above mixes text, random and config-5 launches)
for W in "compress_fast text" "uncompress text" "uncompress_reference text" "compress_fast random" "uncompress random" "compress_ref text" "compress_ref random"; do
  set -- $W
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$1_$2" -o k -- \
    python3 tools/kbench.py --op $1 --data $2 --blocks 10000 --reps ${REPS:-20} > "$OUT/kb_$1_$2.log" 2>&1 || { echo "trace $W failed"; exit 1; }
done
export BLOCKS=10000
bash tools/pmc_run.sh compress_fast "$OUT/pmc_compress" text || exit 1
bash tools/pmc_run.sh uncompress "$OUT/pmc_uncompress" text || exit 1
bash tools/pmc_run.sh compress_fast "$OUT/pmc_compress_random" random || exit 1
bash tools/pmc_run.sh uncompress "$OUT/pmc_uncompress_random" random || exit 1
bash tools/pmc_run.sh compress_fragments "$OUT/pmc_compress_fragments" text || exit 1
bash tools/pmc_run.sh uncompress_reference "$OUT/pmc_uncompress_reference" text || exit 1
python3 tools/pmc_json.py "$OUT" "$OUT/pmc.json" "${COMMIT:-}"
echo profile done
