"""Ablation timing of the super-chunk fast compressor (design tool): the median launch time of the
fast compress of the 10K text blocks, for the library named by SNAPPY_MI355X_LIB (build variants
with -DSC_ABL=bits; their output is not valid and is not checked).

  python tools/sc_abl.py [--blocks 10000] [--reps 20] [--label NAME]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--label", default=os.environ.get("SNAPPY_MI355X_LIB", "default"))
    ap.add_argument("--data", default="text")
    args = ap.parse_args()
    sm = bench.load_package()
    dev = torch.device("cuda", 0)
    blocks = bench.text_blocks(args.blocks, 0x5EED) if args.data == "text" else bench.random_blocks(args.blocks, 0x5EED + 1)
    b = bench.Batch(blocks, dev)
    s = torch.cuda.current_stream()
    for _ in range(3):
        b.compress(sm, "fast")
    ts = []
    for _ in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        b.compress(sm, "fast")
        e1.record(s)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    print("%-40s %s: median %.3f ms, min %.3f ms" % (os.path.basename(args.label), args.data, ts[len(ts) // 2], ts[0]), flush=True)


if __name__ == "__main__":
    main()
