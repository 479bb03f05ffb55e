"""Where a single sm_compress / sm_uncompress call's time goes (design tool, GPU box): medians of
the call on inputs of several sizes beside the floor of the same transfers (pageable host
buffers, torch copies) and an empty launch + synchronize.  python tools/single_call_probe.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def med(fn, n=50):
    fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


def main():
    sm = bench.load_package_cached()
    dev = torch.device("cuda", 0)
    td = os.path.join(ROOT, "tests", "golden", "testdata")
    al = open(os.path.join(td, "alice29.txt"), "rb").read()
    cases = [("tiny 100B", al[:100]), ("4 KiB", al[:4096]), ("tweet", open(os.path.join(td, "sample-tweet.json"), "rb").read()),
             ("64 KiB", al[:65536]), ("html", open(os.path.join(td, "html"), "rb").read()), ("alice29", al),
             ("urls", open(os.path.join(td, "urls.10K"), "rb").read())]
    z = torch.zeros(1, device=dev)
    print("empty launch + sync: %.1f us" % med(lambda: (z.add_(1), torch.cuda.synchronize())))
    for name, data in cases:
        comp = sm.compress(data)
        h = torch.from_numpy(np.frombuffer(comp, np.uint8).copy())
        d = torch.empty(len(data) + 16, dtype=torch.uint8, device=dev)
        hc = torch.empty(len(data), dtype=torch.uint8)
        t_h2d = med(lambda: (d[: len(comp)].copy_(h), torch.cuda.synchronize()))
        t_d2h = med(lambda: (hc.copy_(d[: len(data)]), torch.cuda.synchronize()))
        tc = med(lambda: sm.compress(data))
        tu = med(lambda: sm.uncompress(comp))
        print("%-10s %8d B -> %7d B: compress %7.1f us, uncompress %7.1f us (path %d); H2D(comp) %5.1f us, D2H(out) %5.1f us"
              % (name, len(data), len(comp), tc, tu, sm.last_uncompress_path(), t_h2d, t_d2h))


if __name__ == "__main__":
    main()
