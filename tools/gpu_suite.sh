# GPU suite + a short check script (GPU box): bash tools/gpu_suite.sh <tag> [extra command]
set -u
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc = 0 ] || { grep -E "Error|assert|FAILED" $O/pytest_gpu.log | head -30; exit 1; }
if [ $# -gt 1 ]; then shift; eval "$@"; fi
