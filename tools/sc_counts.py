"""Compressor resync statistics per corpus file from a counting build of sm_compress_sc.hip
(design tool, GPU box): python3 tools/sc_counts.py tools/ablib/lib_sccnt.so -- per super-chunk:
resync rounds (the loop's passes, the last finding nothing to change), lanes rewalking, and
extensions computed (lanes whose last token filled its 16-byte window)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from ab_raw import load, p  # noqa: E402

L, ctx = load(sys.argv[1])
L.sm_diag_sc_counts.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda", 0)
stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
sets = [("bench text", bench.text_blocks(2000, 0x5EED))]
for f in ("alice29.txt", "html", "kppkn.gtb", "geo.protodata", "urls.10K", "smallrandom1.bin"):
    raw = np.frombuffer(open(os.path.join(bench.TESTDATA, f), "rb").read(), np.uint8)
    tiled = np.tile(raw, (2 * bench.BLOCK) // raw.size + 2)
    offs = np.random.default_rng(7).integers(0, tiled.size - bench.BLOCK, 2000)
    sets.append((f, np.ascontiguousarray(np.lib.stride_tricks.sliding_window_view(tiled, bench.BLOCK)[offs])))
for name, blocks in sets:
    B = bench.Batch(blocks, dev)
    c0 = (ctypes.c_ulonglong * 8)()
    L.sm_diag_sc_counts(c0)
    assert L.sm_compress_batch_device(ctx, p(B.d_in), p(B.in_off), p(B.in_len), B.nblk, p(B.d_comp), p(B.comp_off),
                                      p(B.comp_len), 1, stream) == 0
    torch.cuda.synchronize()
    c1 = (ctypes.c_ulonglong * 8)()
    L.sm_diag_sc_counts(c1)
    d = [c1[i] - c0[i] for i in range(8)]
    n = max(d[0], 1)
    print("%-18s super-chunks %7d: resync passes %.2f, rewalking lanes %.1f, extensions %.1f per super-chunk"
          % (name, d[0], d[1] / n, d[2] / n, d[3] / n), flush=True)
