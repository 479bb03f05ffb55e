set -u
bash tools/gpu_base.sh r06_b2 || exit 1
timeout -k 10 500 bash tools/single_call_ab.sh tools/ablib/lib_spin.so tools/ablib/lib_blocksync.so > gpurun_out/r06_b2/sc_ab.log 2>&1 || { echo sc_ab failed; tail gpurun_out/r06_b2/sc_ab.log; exit 1; }
grep -v amdgpu gpurun_out/r06_b2/sc_ab.log
