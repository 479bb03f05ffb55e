"""Block-tail probe (design tool, GPU box): fast-mode compress time per input byte of the bench
text blocks cut to n bytes, for n around multiples of the 15 worker waves' super-chunks.
A block of 60 super-chunks is 4 full rounds of 15 workers; 63 or 64 leave a partial round."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package()
dev = torch.device("cuda", 0)
b = bench.Batch(bench.text_blocks(10000, 0x5EED), dev)
for rnd in range(2):
    for nsc in (30, 32, 45, 48, 60, 61, 63, 64):
        n = 1024 * nsc
        b.in_len.fill_(n)
        ms = bench.kernel_ms(lambda: b.compress(sm, "fast"), 10)
        print("round %d: %2d super-chunks (%5d B): %.4f ms, %.3f ns per KiB-block-byte x 1e3 -> %.2f us per super-chunk-round"
              % (rnd, nsc, n, ms, ms * 1e6 / (10000 * n) * 1e3, ms * 1e3 / (10000 / 256) / nsc), flush=True)
