"""Single-call times of the small benchmark files by decode path and compress split (design
tool, GPU box): median us of sm.uncompress with path 4 on/off and sm.compress with the split
parse on/off.  python3 tools/single_paths.py"""
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
al = open(os.path.join(td, "alice29.txt"), "rb").read()
cases = [("100B", al[:100]), ("1KiB", al[:1024]), ("4KiB", al[:4096]), ("8KiB", al[:8192]), ("16KiB", al[:16384]),
         ("tweet", open(os.path.join(td, "sample-tweet.json"), "rb").read()), ("32KiB", al[:32768]),
         ("64KiB", al[:65536]), ("html", open(os.path.join(td, "html"), "rb").read()),
         ("jpeg", open(os.path.join(td, "fireworks.jpeg"), "rb").read()),
         ("pdf", open(os.path.join(td, "paper-100k.pdf"), "rb").read())]
for name, data in cases:
    comp = sm.compress(data, mode="fast")
    row = []
    for small in (True, False):
        sm.set_small_decode(small)
        assert sm.uncompress(comp) == data
        row.append("u(path4 %s) %.1f [path %d]" % ("on" if small else "off", med(lambda: sm.uncompress(comp)),
                                                   sm.last_uncompress_path()))
    sm.set_small_decode(True)
    for split in (True, False):
        sm.set_split_compress(split)
        assert sm.compress(data, mode="fast") == comp
        row.append("c(split %s) %.1f" % ("on" if split else "off", med(lambda: sm.compress(data, mode="fast"))))
    sm.set_split_compress(True)
    print("%-6s %7d -> %7d: %s" % (name, len(data), len(comp), "  ".join(row)), flush=True)
