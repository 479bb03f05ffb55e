# Section stamps of the fast compressor (design tool; run on the GPU box after tools/gpu_quick.sh)
set -u
O=gpurun_out/${1:-stamps}
mkdir -p $O
SNAPPY_MI355X_LIB=tools/abl/lib_stamp.so timeout -k 10 120 python3 tools/sc_stamps.py > $O/stamps.log 2>&1 || { echo stamps failed; tail $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log
