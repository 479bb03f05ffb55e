# Single-call table for two library builds, alternating on one box (design tool, GPU box):
# tools/single_call_ab.sh libA.so libB.so -> gpurun_out/sc_ab/<n>_<lib>.json
set -u
O=gpurun_out/sc_ab
mkdir -p $O
for r in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    SNAPPY_MI355X_LIB=$L timeout -k 10 200 python3 tools/single_call.py > $O/${r}_$n.json 2> $O/${r}_$n.err || { echo "$L failed"; tail -3 $O/${r}_$n.err; exit 1; }
    python3 - $O/${r}_$n.json $n <<'P'
import json, sys
d = json.load(open(sys.argv[1]))["files"]
print(sys.argv[2], " ".join("%s c%.0f/u%.0f" % (k, v["fast"]["compress_us"], v["fast"]["uncompress_us"]) for k, v in d.items()))
P
  done
done
