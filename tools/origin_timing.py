"""Timing of sm_uncompress on a large stream that is NOT block-structured (copies reach into
earlier 64 KiB blocks), which takes the origin-pointer parallel path (design tool, GPU box)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from streams import build, random_ops  # noqa: E402


def main():
    sm = bench.load_package()
    rng = np.random.default_rng(5)
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    t0 = time.perf_counter()
    s, e = build(random_ops(rng, mb << 20, max_off=65535, near=30_000))
    print("built %d -> %d B in %.1f s" % (len(e), len(s), time.perf_counter() - t0), flush=True)
    assert sm.uncompress(s) == e
    print("path", sm.last_uncompress_path(), flush=True)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        out = sm.uncompress(s)
        ts.append(time.perf_counter() - t0)
    assert out == e
    print("sm_uncompress (host buffers, PCIe included): %.1f ms = %.2f GB/s uncompressed" % (
        min(ts) * 1e3, len(e) / min(ts) / 1e9), flush=True)


if __name__ == "__main__":
    main()
