"""Single-call uncompress of long-chain streams (runs: every copy byte's origin pointer is a long
chain for path 4's resolve launches), library from SNAPPY_MI355X_LIB (design tool, GPU box):
python3 tools/chain_case.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package_cached()
rng = np.random.default_rng(5)
cases = {
    "zeros_64K": bytes(65536),
    "zeros_1M": bytes(1 << 20),
    "zeros_8M": bytes(8 << 20),
    "period3_1M": (b"abc" * 350000)[: 1 << 20],
    "runs_1M": np.repeat(rng.integers(0, 256, 4096, dtype=np.uint8), 256).tobytes(),
}
row = []
for name, data in cases.items():
    comp = sm.compress(data, mode="fast")
    assert sm.uncompress(comp) == data
    ts = []
    for _ in range(30):
        t0 = time.perf_counter()
        sm.uncompress(comp)
        ts.append(time.perf_counter() - t0)
    row.append("%s p%d %.0f" % (name, sm.last_uncompress_path(), float(np.median(ts)) * 1e6))
print(os.path.basename(os.environ.get("SNAPPY_MI355X_LIB", "in-tree")), " ".join(row), flush=True)
