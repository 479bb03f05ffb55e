"""Fast-mode batched compress rate per corpus file (design tool, GPU box): 2,000 64 KiB windows
of each file (tiled, seeded offsets), timed like the bench; explains config 5's mix rate."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package()
dev = torch.device("cuda", 0)
nb = 2000
for f in bench.ROUNDTRIP_FILES:
    raw = np.frombuffer(open(os.path.join(bench.TESTDATA, f), "rb").read(), np.uint8)
    tiled = np.tile(raw, (2 * bench.BLOCK) // raw.size + 2)
    rng = np.random.default_rng(7)
    offs = rng.integers(0, tiled.size - bench.BLOCK, nb)
    blocks = np.ascontiguousarray(np.lib.stride_tricks.sliding_window_view(tiled, bench.BLOCK)[offs])
    b = bench.Batch(blocks, dev)
    ms = bench.kernel_ms(lambda: b.compress(sm, "fast"), 10)
    msd = bench.kernel_ms(lambda: b.uncompress(sm), 10)
    print("%-18s %7d B: compress %6.1f GB/s  uncompress %6.1f GB/s  ratio %.3f  (%.3f / %.3f ms per 2000 blocks)"
          % (f, raw.size, b.in_bytes / ms / 1e6, b.in_bytes / msd / 1e6, b.comp_bytes() / b.in_bytes, ms, msd), flush=True)
