#!/bin/bash
# Copies a round's GPU evidence (tools/round_all.sh <round> output) into profiles/ (run here).
set -e
R=$1
G=gpurun_out
cp $G/$R/bench.json profiles/${R}_bench.json
tail -3 $G/$R/pytest_gpu.log > profiles/${R}_pytest_gpu.log
cp $G/${R}_prof/trace/bench_kernel_stats.csv profiles/${R}_bench_kernel_stats.csv
for W in compress_fast_text uncompress_text compress_fast_random uncompress_random compress_ref_text compress_ref_random; do
  cp $G/${R}_prof/trace_$W/k_kernel_stats.csv profiles/${R}_kernel_stats_$W.csv
done
cp $G/${R}_prof/pmc.json profiles/${R}_pmc.json
[ -f $G/$R/fast_sizes.txt ] && cp $G/$R/fast_sizes.txt profiles/${R}_fast_sizes.txt
echo collected
