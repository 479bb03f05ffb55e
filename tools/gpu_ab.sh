# A/B of library builds in tools/ablib on the GPU box: bash tools/gpu_ab.sh <tag> "<ab_raw args>" lib1 lib2 ...
set -u
O=gpurun_out/$1; shift
ARGS=$1; shift
mkdir -p $O
timeout -k 10 400 python3 tools/ab_raw.py $ARGS "$@" > $O/ab.log 2>&1 || { echo ab failed; tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log | tail -25
