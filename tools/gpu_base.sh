# Round-6 baseline on the GPU box: GPU suite, then kernel timings of the headline kernels.
set -u
O=gpurun_out/${1:-base}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc = 0 ] || { grep -E "Error|assert|FAILED" $O/pytest_gpu.log | head -30; exit 1; }
for op in compress_fast uncompress; do
  timeout -k 10 120 python3 tools/kbench.py --op $op --blocks 10000 --reps 20 >> $O/t.log 2>&1 || { echo kbench failed; tail $O/t.log; exit 1; }
done
timeout -k 10 120 python3 tools/kbench.py --op compress_fragments --reps 10 >> $O/t.log 2>&1 || { echo kbench failed; tail $O/t.log; exit 1; }
grep -v amdgpu.ids $O/t.log
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json | head -c 3000
