set -u
O=gpurun_out/r06_b11; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc = 0 ] || { grep -E "Error|assert|FAILED" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 120 python3 tools/pyoverhead.py > $O/pyo.txt 2>&1 || { tail $O/pyo.txt; exit 1; }
timeout -k 10 200 python3 tools/single_paths.py > $O/paths.txt 2> $O/paths.err || { echo paths failed; tail $O/paths.err; exit 1; }
grep -v amdgpu.ids $O/pyo.txt; cat $O/paths.txt
