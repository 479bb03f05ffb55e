"""Debug driver: compress a few text blocks with the fast compressor and print out_len (hand-off
error marks 0xfff0000x) and the time."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    sm = bench.load_package()
    dev = torch.device("cuda", 0)
    b = bench.Batch(bench.text_blocks(nb, 0x5EED), dev)
    t0 = time.time()
    b.compress(sm, "fast")
    torch.cuda.synchronize()
    print("time %.3f s" % (time.time() - t0), flush=True)
    print([hex(x & 0xffffffff) for x in b.comp_len.cpu().tolist()[:16]], flush=True)
    print("roundtrip", b.verify(), flush=True)


if __name__ == "__main__":
    main()
