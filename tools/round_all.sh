# Round-end evidence on the GPU box: GPU suite, bench (with extras), kernel traces and PMC passes.
# Usage: bash tools/round_all.sh <round>   -> gpurun_out/<round>/..., gpurun_out/<round>_prof/...
set -u
R=$1
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc = 0 ] || { echo "pytest rc $rc"; exit 1; }
timeout -k 10 400 python bench.py --extras > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
[ "${SKIP_PROF:-0}" = 1 ] || bash tools/profile_round.sh $R || exit 1
