"""Run-to-run determinism of the fast compressor on the bench workload (design tool, GPU box).

  python tools/determinism.py [--blocks 10000] [--reps 8] [--mode fast|dense]
Compresses the same device-resident batch `reps` times and compares every output byte and size
with the first launch, then decodes the first launch on the GPU and checks the round trip.
Used for the round-1 g22 incident (invalid, run-to-run different fast-mode streams at 128 VGPRs):
a race or a miscompile shows up here as a mismatch between launches.
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
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--mode", default="fast")
    ap.add_argument("--data", default="text")
    args = ap.parse_args()
    sm = bench.load_package()
    dev = torch.device("cuda", 0)
    blocks = bench.text_blocks(args.blocks, 0x5EED) if args.data == "text" else bench.random_blocks(args.blocks, 0x5EED + 1)
    b = bench.Batch(blocks, dev)
    b.d_comp.fill_(0)
    b.compress(sm, args.mode)
    torch.cuda.synchronize()
    ref, ref_len = b.d_comp.clone(), b.comp_len.clone()
    bad = 0
    for i in range(args.reps):
        b.d_comp.fill_(0x5A if i % 2 else 0)
        b.compress(sm, args.mode)
        torch.cuda.synchronize()
        same_len = bool(torch.equal(b.comp_len, ref_len))
        # compare only the bytes of each stream (slot tails are never written)
        mism = 0
        if same_len:
            nb = b.comp_len.to(torch.int64)
            idx = torch.arange(bench.SLOT, device=dev)[None, :] < nb[:, None]
            a1 = b.d_comp.view(-1, bench.SLOT)[idx]
            a0 = ref.view(-1, bench.SLOT)[idx]
            mism = int((a1 != a0).sum())
        print("launch %d: sizes %s, differing bytes %d" % (i + 1, "equal" if same_len else "DIFFER", mism), flush=True)
        bad += (not same_len) or mism > 0
    b.d_comp.copy_(ref)
    b.comp_len.copy_(ref_len)
    ok = b.verify()
    print("mode %s: %d/%d launches identical to the first; round trip of the first: %s" % (
        args.mode, args.reps - bad, args.reps, ok))
    sys.exit(0 if ok and bad == 0 else 1)


if __name__ == "__main__":
    main()
