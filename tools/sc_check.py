"""Quick GPU check of the fast compressor (development tool): corpus round trips through the oracle,
sizes against reference mode, the 10K-block bench batches (text, random) with their round trip on
the GPU decoder, and launch timing.

  python tools/sc_check.py [--blocks 10000] [--reps 10]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench  # noqa: E402
import oracle as O  # noqa: E402

FILES = ["alice29.txt", "asyoulik.txt", "html", "html_x_4", "kppkn.gtb", "lcet10.txt", "fireworks.jpeg",
         "geo.protodata", "paper-100k.pdf", "plrabn12.txt", "urls.10K", "random1.bin", "random2.bin",
         "random3.bin", "smallrandom1.bin", "sample-tweet.json"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--mode", default="fast")
    ap.add_argument("--skip-corpus", action="store_true")
    args = ap.parse_args()
    sm = bench.load_package()
    print("lib", sm.version(), flush=True)
    if not args.skip_corpus:
        worst = 0.0
        for f in FILES:
            data = open(os.path.join(bench.TESTDATA, f), "rb").read()
            c = sm.compress(data, mode=args.mode, device=0)
            ok = O.uncompress(c) == data
            ref = len(O.compress(data))
            worst = max(worst, len(c) / ref)
            print("%-18s n=%7d fast=%7d ref=%7d x%.4f %s" % (f, len(data), len(c), ref, len(c) / ref, "ok" if ok else "FAIL"),
                  flush=True)
            assert ok, f
        print("worst size vs reference: x%.4f" % worst, flush=True)
    dev = torch.device("cuda", 0)
    for kind in ("text", "random"):
        blocks = bench.text_blocks(args.blocks, 0x5EED) if kind == "text" else bench.random_blocks(args.blocks, 0x5EED + 1)
        b = bench.Batch(blocks, dev)
        b.compress(sm, args.mode)
        torch.cuda.synchronize()
        ok = b.verify()
        ratio = float(b.comp_bytes()) / (args.blocks * bench.BLOCK)
        # a sample through the oracle
        cl = b.comp_len.cpu().numpy()
        out = b.d_comp.cpu().numpy()
        oo = b.comp_off.cpu().numpy()
        nbad = 0
        for i in range(0, args.blocks, max(1, args.blocks // 50)):
            s = bytes(out[oo[i]:oo[i] + cl[i]])
            if O.uncompress(s) != blocks[i].tobytes():
                nbad += 1
        t0 = time.perf_counter()
        for _ in range(args.reps):
            b.compress(sm, args.mode)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        print("%s: compress %.3f ms (%.1f GB/s in), ratio %.4f, gpu roundtrip %s, oracle sample bad %d" % (
            kind, dt * 1e3, args.blocks * bench.BLOCK / dt / 1e9, ratio, ok, nbad), flush=True)
        assert ok and nbad == 0


if __name__ == "__main__":
    main()
