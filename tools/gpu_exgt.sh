# Reference-mode table placement A/B (design tool; GPU box): LDS (shipped) vs global-memory table
timeout -k 5 60 tools/abl/gx
timeout -k 10 300 python3 tools/exact_bench.py --blocks 10000 --check 2000 2>&1 | grep -v amdgpu.ids
SNAPPY_MI355X_LIB=tools/abl/lib_exgt.so timeout -k 10 300 python3 tools/exact_bench.py --blocks 10000 --check 10000 2>&1 | grep -v amdgpu.ids
