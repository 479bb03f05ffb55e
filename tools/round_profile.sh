#!/bin/bash
# Round-end measurement on the GPU box: GPU tests, bench (with extras), rocprofv3 kernel
# trace + stats of the bench command, PMC traffic passes for both hot kernels.
# Usage: tools/round_profile.sh <round-tag>
set -u
R=${1:-r01}
OUT=gpurun_out/$R
mkdir -p $OUT
timeout -k 10 400 python -m pytest tests -m gpu -q > $OUT/pytest_gpu.log 2>&1; echo "pytest exit $?" >> $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py --extras > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o $R -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $OUT/trace.log 2>&1 || { echo trace failed; tail $OUT/trace.log; exit 1; }
BLOCKS=10000 tools/pmc_run.sh compress_fast $OUT/pmc_compress > $OUT/pmc_compress.log 2>&1 || exit 1
BLOCKS=10000 tools/pmc_run.sh uncompress $OUT/pmc_uncompress > $OUT/pmc_uncompress.log 2>&1 || exit 1
python3 tools/pmc_json.py $OUT $OUT/pmc.json > $OUT/pmc_json.log 2>&1
python3 tools/pmc_summary.py $OUT/pmc_compress k_compress > $OUT/pmc_compress.txt 2>&1
python3 tools/pmc_summary.py $OUT/pmc_uncompress k_decompress > $OUT/pmc_uncompress.txt 2>&1
echo done
