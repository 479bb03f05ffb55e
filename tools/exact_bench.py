"""Reference-mode (byte-identical) compressor: GPU time and full-batch byte parity against the
oracle (design tool, GPU box).  SNAPPY_MI355X_LIB selects a diagnostic build.
  python3 tools/exact_bench.py [--blocks 10000] [--check 10000]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=10000)
    ap.add_argument("--check", type=int, default=10000, help="blocks compared byte-for-byte with the oracle")
    args = ap.parse_args()
    import torch
    import oracle as O
    sm = bench.load_package()
    dev = torch.device("cuda", 0)
    for kind in ("text", "random"):
        blocks = bench.text_blocks(args.blocks, 0x5EED) if kind == "text" else bench.random_blocks(args.blocks, 0x5EED + 1)
        b = bench.Batch(blocks, dev)
        ms = bench.kernel_ms(lambda: b.compress(sm, "reference"), 3)
        clen = b.comp_len.cpu().numpy().astype(np.uint32)
        comp = b.d_comp.cpu().numpy()
        n = min(args.check, args.blocks)
        if n == 0:
            print("%s: %.3f ms  %.3f GB/s" % (kind, ms, args.blocks * bench.BLOCK / (ms * 1e-3) / 1e9), flush=True)
            continue
        inp = np.ascontiguousarray(blocks[:n]).reshape(-1)
        o_comp = np.zeros(n * bench.SLOT, dtype=np.uint8)
        o_len = np.zeros(n, dtype=np.uint32)
        O.compress_batch(inp, np.arange(n, dtype=np.uint64) * bench.BLOCK, np.full(n, bench.BLOCK, np.uint32), o_comp,
                         np.arange(n, dtype=np.uint64) * bench.SLOT, o_len, compat=False, nthreads=16)
        bad = [i for i in range(n) if o_len[i] != clen[i] or
               not np.array_equal(comp[i * bench.SLOT:i * bench.SLOT + clen[i]], o_comp[i * bench.SLOT:i * bench.SLOT + o_len[i]])]
        print("%s: %.3f ms  %.3f GB/s  ratio %.5f  byte-identical %d/%d%s" % (
            kind, ms, args.blocks * bench.BLOCK / (ms * 1e-3) / 1e9, clen[:args.blocks].sum() / (args.blocks * bench.BLOCK),
            n - len(bad), n, (" first bad %s" % bad[:5]) if bad else ""), flush=True)
        print("  roundtrip", b.verify(), flush=True)


if __name__ == "__main__":
    main()
