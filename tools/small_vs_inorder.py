"""Single-call uncompress of each corpus file's fast stream with path 4 (small streams on the device)
enabled and disabled (then path 0/1), same process (design tool, GPU box):
python3 tools/small_vs_inorder.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package_cached()
TD = os.path.join(ROOT, "tests", "golden", "testdata")


def med(fn, n=60):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


for f in sorted(os.listdir(TD)):
    data = open(os.path.join(TD, f), "rb").read()
    if len(data) < 4096:
        continue
    comp = sm.compress(data, mode="fast")
    row = []
    for en in (1, 0):
        sm.set_small_decode(en)
        assert sm.uncompress(comp) == data
        p = sm.last_uncompress_path()
        row.append("path %d %7.1f us" % (p, med(lambda: sm.uncompress(comp))))
    sm.set_small_decode(1)
    print("%-22s %8d B  body/out %.3f   %s | %s" % (f, len(data), len(comp) / len(data), row[0], row[1]), flush=True)
