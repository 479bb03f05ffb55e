set -u
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for W in "compress_fast text" "uncompress text"; do
  set -- $W
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$1_$2" -o k -- python3 tools/kbench.py --op $1 --data $2 --blocks 10000 --reps 20 > "$O/kb_$1_$2.log" 2>&1 || { echo "trace $W failed"; exit 1; }
  cat $O/kb_$1_$2.log
done
echo done
