"""Kernel driver for profiling (rocprofv3 --kernel-trace / --pmc): runs one codec kernel R
times on the bench workload (text or random 64 KiB blocks), device-resident.

  python tools/kbench.py --op compress_fast|compress_ref|uncompress|uncompress_reference --blocks 2000 --reps 5 [--data random]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="compress_fast")
    ap.add_argument("--blocks", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--data", default="text")
    args = ap.parse_args()
    sm = bench.load_package()
    dev = torch.device("cuda", 0)
    print("library", sm.version())
    if args.op in ("compress_fragments", "uncompress_fragments"):
        return fragments(sm, dev, args)
    blocks = bench.text_blocks(args.blocks, 0x5EED) if args.data == "text" else bench.random_blocks(args.blocks, 0x5EED + 1)
    b = bench.Batch(blocks, dev)
    # uncompress_reference: the decode of the reference-mode (Snappy.jl byte-identical) streams
    b.compress(sm, "reference" if args.op == "uncompress_reference" else "fast")
    torch.cuda.synchronize()
    ops = {
        "compress_fast": lambda: b.compress(sm, "fast"),
        "compress_dense": lambda: b.compress(sm, "dense"),
        "compress_ref": lambda: b.compress(sm, "reference"),
        "uncompress": lambda: b.uncompress(sm),
        "uncompress_reference": lambda: b.uncompress(sm),
    }
    fn = ops[args.op]
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.reps
    nbytes = args.blocks * bench.BLOCK
    print("%s %s: %.3f ms/launch, %.2f GB/s (uncompressed bytes), ratio %.4f" % (
        args.op, args.data, dt * 1e3, nbytes / dt / 1e9, float(b.comp_len.sum()) / nbytes))
    if not args.op.startswith("uncompress"):
        b.uncompress(sm)
    print("roundtrip ok:", b.verify())


def fragments(sm, dev, args):
    """Config 5 (bench.py `large`): the 644 MiB stream's 10,304 fragments on one GPU."""
    big = bench.large_corpus()
    nfrag = (big.size + bench.BLOCK - 1) // bench.BLOCK
    sh = bench.StreamShard(big, 0, nfrag, dev)
    sh.compress(sm)
    sh.index(bench.load_dist(), 0, 1)  # (world 1, no process group: the scan alone)
    sh.place(sm)  # (the fragments decode from the placed stream)
    torch.cuda.synchronize()
    fn = (lambda: sh.compress(sm)) if args.op == "compress_fragments" else (lambda: sh.uncompress(sm))
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.reps
    print("%s: %.3f ms/launch, %.2f GB/s (uncompressed bytes)" % (args.op, dt * 1e3, sh.in_bytes / dt / 1e9))
    print("roundtrip ok:", sh.verify(sm))


if __name__ == "__main__":
    main()
