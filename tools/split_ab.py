"""Single-call compress latency of one file (design tool, GPU box): median of 300 calls.
SNAPPY_MI355X_LIB=tools/abl/lib_x.so python3 tools/split_ab.py html"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package_cached()
for f in sys.argv[1:]:
    raw = open(os.path.join(ROOT, "tests", "golden", "testdata", f), "rb").read()
    sm.compress(raw)
    ts = []
    for _ in range(300):
        t0 = time.perf_counter()
        sm.compress(raw)
        ts.append(time.perf_counter() - t0)
    print("%-20s %s %7.1f us" % (f, os.environ.get("SNAPPY_MI355X_LIB", "default")[-20:], np.median(ts) * 1e6))
