# Round-5: GPU suite, batch A/B of the product against the previous commit's build, single-call A/B
# against round 4 (design tool, GPU box).
set -u
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest rc $rc"; exit 1; }
timeout -k 10 300 python tools/ab_raw.py --rounds 3 ${ABLIBS:-tools/ablib/lib_r05fence.so} snappy.jl_amd/libsnappy_mi355x.so > $O/ab.log 2>&1 \
  || { echo "ab rc $?"; tail -5 $O/ab.log; exit 1; }
grep -v "^round" $O/ab.log
bash tools/single_call_ab.sh tools/ablib/lib_r04.so snappy.jl_amd/libsnappy_mi355x.so
