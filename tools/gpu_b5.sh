# parts/single-call GPU tests, then single-call paths on the current build
set -u
O=gpurun_out/r06_b5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "parts or single or pinned or split or small" > $O/pytest_sub.log 2>&1; rc=$?
tail -3 $O/pytest_sub.log
[ $rc = 0 ] || { grep -E "Error|assert|FAILED" $O/pytest_sub.log | head -30; exit 1; }
timeout -k 10 200 python3 tools/single_paths.py > $O/paths.txt 2> $O/paths.err || { echo paths failed; tail $O/paths.err; exit 1; }
cat $O/paths.txt
