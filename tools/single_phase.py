"""Phase times of single calls (design tool, GPU box): loads a -DSM_HOST_TRACE build of the
library (make -C snappy.jl_amd/csrc SM_VARIANT=1 OUT=../libsnappy_mi355x_trace.so OBJ=build_trace
EXTRA=-DSM_HOST_TRACE), whose host entry points print a synchronised timestamp per phase on stderr.
python3 tools/single_phase.py fireworks.jpeg:u sample-tweet.json:c ..."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package_cached()
sm._lib = sm.load_library(os.path.join(ROOT, "snappy.jl_amd", "libsnappy_mi355x_trace.so"))
for spec in sys.argv[1:]:
    f, op = spec.split(":")
    mode = "fast"
    if "/" in op:
        op, mode = op.split("/")
    data = open(os.path.join(ROOT, "tests", "golden", "testdata", f), "rb").read()
    comp = sm.compress(data, mode=mode)
    for _ in range(20):  # warm
        sm.uncompress(comp) if op == "u" else sm.compress(data, mode=mode)
    sys.stderr.flush()
    print("=== %s %s (%s): %d -> %d B" % (f, "uncompress" if op == "u" else "compress", mode, len(data), len(comp)),
          file=sys.stderr, flush=True)
    for _ in range(3):
        t0 = time.perf_counter()
        sm.uncompress(comp) if op == "u" else sm.compress(data, mode=mode)
        print("  total %.1f us (path %d)" % ((time.perf_counter() - t0) * 1e6, sm.last_uncompress_path()),
              file=sys.stderr, flush=True)
