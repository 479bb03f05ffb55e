"""Decoder section timing from in-kernel s_memtime stamps (design tool, GPU box).

Build the diagnostic library, then run:
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DSM_STAMP=1 -o tools/abl/lib_stamp.so \
      snappy.jl_amd/csrc/sm_*.hip
  SNAPPY_MI355X_LIB=tools/abl/lib_stamp.so python3 tools/stamp_run.py [--data text|random]
  ... --op compress_fast: the fast compressor's per-round sections instead.
Decoder sections (per wave, summed over all streams): 0 flush + ring management, 1 tag walk,
2 per-tag decode + error checks, 3 long literals, 8 the execution round, 4 the in-order tail
(copies whose source is in the batch), 5 big literals; counters 6 = batches, 7 = rounds +
in-order tags, 9 = in-order tags.
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

NAMES = ["ring+flush", "walk", "decode", "longlit", "in-order tail", "big literals", "", "", "round"]
CNAMES = ["", "", "", "parse (all chunks)", "barrier wait", "layout", "emission", "tail"]
INAMES = ["inserter: inserts", "inserter: barrier wait"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=4000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--data", default="text")
    ap.add_argument("--op", default="uncompress", choices=["uncompress", "compress_fast", "compress_ref"])
    args = ap.parse_args()
    if args.op == "compress_fast":
        return compress_stamps(args)
    if args.op == "compress_ref":
        return exact_stamps(args)
    sm = bench.load_package()
    lib = sm.lib()
    fn = lib.sm_debug_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    dev = torch.device("cuda", 0)
    blocks = bench.text_blocks(args.blocks, 0x5EED) if args.data == "text" else bench.random_blocks(args.blocks, 0x5EED + 1)
    b = bench.Batch(blocks, dev)
    b.compress(sm, "fast")
    b.uncompress(sm)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 10)()
    fn(buf, 1)
    for _ in range(args.reps):
        b.uncompress(sm)
    torch.cuda.synchronize()
    fn(buf, 1)
    v = list(buf)
    tot = sum(v[:6]) + v[8]
    batches, rounds = v[6], v[7]
    print("data %s: %d batches (%.1f per block), %d rounds (%.2f per batch), %.2f in-order tags per batch" % (
        args.data, batches, batches / args.blocks / args.reps, rounds, rounds / max(batches, 1),
        v[9] / max(batches, 1)))
    for i, nme in enumerate(NAMES):
        if nme:
            print("  %-18s %5.1f%%  %8.0f cycles/batch" % (nme, 100.0 * v[i] / tot, v[i] / max(batches, 1)))
    print("  total              %8.0f cycles/batch" % (tot / max(batches, 1)))
    print("roundtrip ok:", b.verify())


def compress_stamps(args):
    sm = bench.load_package()
    fn = sm.lib().sm_debug_stamps_c
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    dev = torch.device("cuda", 0)
    blocks = bench.text_blocks(args.blocks, 0x5EED) if args.data == "text" else bench.random_blocks(args.blocks, 0x5EED + 1)
    b = bench.Batch(blocks, dev)
    b.compress(sm, "fast")
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 28)()
    fn(buf, 1)
    for _ in range(args.reps):
        b.compress(sm, "fast")
    torch.cuda.synchronize()
    fn(buf, 1)
    v = list(buf)
    rounds, irounds = v[11], v[10]
    tot = sum(v[:8])
    print("compress_fast %s: %d parsed chunks, %d inserter rounds" % (args.data, rounds, irounds))
    for i, nme in enumerate(CNAMES):
        if nme:
            print("  %-24s %5.1f%%  %7.0f cycles/chunk" % (nme, 100.0 * v[i] / tot, v[i] / max(rounds, 1)))
    print("  total (parse waves)      %7.0f cycles/chunk" % (tot / max(rounds, 1)))
    itot = v[8] + v[9]
    for i, nme in enumerate(INAMES):
        print("  %-24s %5.1f%%  %7.0f cycles/round" % (nme, 100.0 * v[8 + i] / max(itot, 1), v[8 + i] / max(irounds, 1)))
    print("  barrier wait per wave index (cycles/round): " +
          " ".join("%d" % (v[12 + w] / max(irounds, 1)) for w in range(16)))


XNAMES = ["search", "flush (emission)", "copy round", "token+hash+table", "loop top", "remainder"]


def exact_stamps(args):
    sm = bench.load_package()
    fn = sm.lib().sm_debug_stamps_x
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    dev = torch.device("cuda", 0)
    blocks = bench.text_blocks(args.blocks, 0x5EED) if args.data == "text" else bench.random_blocks(args.blocks, 0x5EED + 1)
    b = bench.Batch(blocks, dev)
    buf = (ctypes.c_ulonglong * 8)()
    b.compress(sm, "reference")
    torch.cuda.synchronize()
    fn(buf, 1)
    b.compress(sm, "reference")
    torch.cuda.synchronize()
    fn(buf, 1)
    v = list(buf)
    copies = v[6]
    tot = sum(v[:6])
    print("compress_ref %s: %d copy steps (%.0f per block), %d probe steps (%.0f per block)" % (
        args.data, copies, copies / args.blocks, v[7], v[7] / args.blocks))
    for i, nme in enumerate(XNAMES):
        print("  %-24s %5.1f%%  %7.0f cycles/copy" % (nme, 100.0 * v[i] / tot, v[i] / max(copies, 1)))


if __name__ == "__main__":
    main()
