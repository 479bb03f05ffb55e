# Quick check on the GPU box: the GPU suite, then fast-compress timing (text, random) and a round trip
set -u
O=gpurun_out/${1:-quick}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -15 $O/pytest_gpu.log
[ $rc = 0 ] || { echo "pytest rc $rc"; exit 1; }
timeout -k 10 120 python3 tools/sc_abl.py --label head > $O/t.log 2>&1 && timeout -k 10 120 python3 tools/sc_abl.py --label head --data random >> $O/t.log 2>&1 || { echo timing failed; tail $O/t.log; exit 1; }
timeout -k 10 120 python3 tools/kbench.py --op compress_fast --blocks 10000 --reps 20 >> $O/t.log 2>&1 && timeout -k 10 120 python3 tools/kbench.py --op uncompress --blocks 10000 --reps 20 >> $O/t.log 2>&1 || { echo kbench failed; tail $O/t.log; exit 1; }
grep -v amdgpu.ids $O/t.log
