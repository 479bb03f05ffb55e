# round-end sequence on one box: GPU suite, profiles (kernel traces + PMC), then the bench lines
# against the fresh PMC file (copied into this box's tree first, so the line's traffic is of the
# same build)
set -u
R=${1:-r06}
mkdir -p gpurun_out/${R}_final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${R}_final/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/${R}_final/pytest_gpu.log
[ $rc = 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${R}_final/pytest_gpu.log | head -30; exit 1; }
rm -rf gpurun_out/${R}_prof
COMMIT=${COMMIT:-} bash tools/profile_round.sh $R || exit 1
cp gpurun_out/${R}_prof/pmc.json profiles/${R}_pmc.json
bash tools/gpu_bench.sh ${R}_bench > /dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/${R}_bench/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['traffic_source']['same_build'])"
