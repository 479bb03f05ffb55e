#!/bin/bash
# A/B of the final-round inserter parse (SM_FAST_LASTINS): kbench on the 10K bench blocks,
# alternating the shipped library and a -DSM_FAST_LASTINS=0 build, then the GPU suite.
set -u
O=gpurun_out/lastins; mkdir -p $O
for i in 1 2; do
  for L in snappy.jl_amd/lib_nolastins.so snappy.jl_amd/libsnappy_mi355x.so; do
    for D in text random; do
      SNAPPY_MI355X_LIB=$PWD/$L timeout -k 10 120 python tools/kbench.py --op compress_fast --data $D --blocks 10000 --reps 30 > $O/kb.tmp 2>&1 || { cat $O/kb.tmp; exit 1; }
      echo "$L $D $(grep -v amdgpu.ids $O/kb.tmp | tr '\n' ' ')" >> $O/ab.txt
    done
  done
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
