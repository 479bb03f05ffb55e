"""Python-side cost of a single call (design tool, GPU box): sm.compress / sm.uncompress against
the raw C call with preallocated buffers, median us of 400 calls."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package_cached()


def med(fn, n=400):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


td = os.path.join(ROOT, "tests", "golden", "testdata")
L = sm.lib()
ctx = sm.context(0)
for f in ("sample-tweet.json", "fireworks.jpeg", "html"):
    data = open(os.path.join(td, f), "rb").read()
    comp = sm.compress(data, mode="fast")
    src = np.frombuffer(data, np.uint8)
    csrc = np.frombuffer(comp, np.uint8)
    out = np.empty(sm.maxlength_compressed(len(data)), np.uint8)
    dec = np.empty(len(data), np.uint8)
    ol = ctypes.c_size_t(0)

    def rc():
        ol.value = out.size
        return L.sm_compress(ctx, src.ctypes.data, src.size, out.ctypes.data, ctypes.byref(ol), 1)

    def ru():
        ol.value = dec.size
        return L.sm_uncompress(ctx, csrc.ctypes.data, csrc.size, dec.ctypes.data, ctypes.byref(ol))

    assert rc() == 0 and ru() == 0
    print("%-18s compress: wrapper %.1f us, raw C %.1f us | uncompress: wrapper %.1f us, raw C %.1f us" % (
        f, med(lambda: sm.compress(data, mode="fast")), med(rc), med(lambda: sm.uncompress(comp)), med(ru)), flush=True)
