# round-3 session: corpus check, GPU suite + timings of the in-tree library, corpus sizes, compress A/B
# against the variants given, decompress A/B against $DEC_LIBS
set -u
mkdir -p gpurun_out/s3b
timeout -k 10 180 python3 tools/sc_check.py --blocks 2000 --reps 3 > gpurun_out/s3b/sc_check.log 2>&1 || { echo sc_check failed; tail -20 gpurun_out/s3b/sc_check.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s3b/sc_check.log | tail -25
bash tools/gpu_quick.sh s3b || exit 1
timeout -k 10 120 python3 tools/fast_sizes.py > gpurun_out/s3b/sizes.txt 2>&1 || { echo sizes failed; tail gpurun_out/s3b/sizes.txt; exit 1; }
tail -3 gpurun_out/s3b/sizes.txt
bash tools/gpu_ab.sh s3b_ab "$@" || exit 1
[ -n "${DEC_LIBS:-}" ] && OP=uncompress bash tools/gpu_ab.sh s3b_abd $DEC_LIBS
