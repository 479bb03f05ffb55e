set -u
bash tools/gpu_quick.sh q8 || exit 1
timeout -k 10 120 python3 tools/kbench.py --op compress_dense --blocks 10000 --reps 20 2>&1 | grep -v amdgpu.ids
