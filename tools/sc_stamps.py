"""Section timing of the super-chunk fast compressor from in-kernel s_memtime stamps (design tool).

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-strict-aliasing -fPIC -shared -DSM_STAMP=1 \\
      -o tools/abl/lib_stamp.so snappy.jl_amd/csrc/sm_*.hip
  SNAPPY_MI355X_LIB=tools/abl/lib_stamp.so python3 tools/sc_stamps.py [--data text|random]
Sections are per wave, summed over all waves and blocks, shown per super-chunk.
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

NAMES = ["A hash", "B token wait", "B exchange", "C verify", "D walks+resync", "E sizes", "F base wait",
         "G emission", "writer: wait for a slot", "writer: copy-out"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=4000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--data", default="text")
    args = ap.parse_args()
    sm = bench.load_package()
    fn = sm.lib().sm_debug_stamps_sc
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    dev = torch.device("cuda", 0)
    blocks = bench.text_blocks(args.blocks, 0x5EED) if args.data == "text" else bench.random_blocks(args.blocks, 0x5EED + 1)
    b = bench.Batch(blocks, dev)
    b.compress(sm, "fast")
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 12)()
    fn(buf, 1)
    for _ in range(args.reps):
        b.compress(sm, "fast")
    torch.cuda.synchronize()
    fn(buf, 1)
    v = list(buf)
    nsc = max(v[11], 1)
    tot = sum(v[:8])
    print("data %s: %d super-chunks, %.2f resync iterations each" % (args.data, nsc, v[10] / nsc))
    for i, nme in enumerate(NAMES):
        print("  %-28s %5.1f%%  %8.0f cycles/super-chunk" % (nme, 100.0 * v[i] / tot if i < 8 else 0.0, v[i] / nsc))
    print("  total (worker sections)      %8.0f cycles/super-chunk (wave time)" % (tot / nsc))
    print("roundtrip ok:", b.verify())


if __name__ == "__main__":
    main()
