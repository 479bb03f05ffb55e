"""Decoder batch statistics from a counting build of sm_decompress.hip (design tool, GPU box):
python3 tools/dec_counts.py tools/ablib/lib_cnt.so [text|large|reference]
The build exports sm_diag_counts (device counters: batches, tags left to the in-order loop, of
those with offset < 16, of those whose source precedes the first pending tag, batch tags, batches
with an in-order tail, 16-byte passes)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from ab_raw import load, p  # noqa: E402

L, ctx = load(sys.argv[1])
data = sys.argv[2] if len(sys.argv) > 2 else "text"
L.sm_diag_counts.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda", 0)
blocks = bench.large_corpus().reshape(-1, bench.BLOCK) if data == "large" else bench.text_blocks(10000, 0x5EED)
B = bench.Batch(blocks, dev)
stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
mode = 0 if data == "reference" else 1
assert L.sm_compress_batch_device(ctx, p(B.d_in), p(B.in_off), p(B.in_len), B.nblk, p(B.d_comp), p(B.comp_off),
                                  p(B.comp_len), mode, stream) == 0
torch.cuda.synchronize()
c0 = (ctypes.c_ulonglong * 8)()
L.sm_diag_counts(c0)
assert L.sm_uncompress_batch_device(ctx, p(B.d_comp), p(B.comp_off), p(B.comp_len), B.nblk, p(B.d_dec), p(B.in_off),
                                    p(B.dec_cap), p(B.dec_len), p(B.status), stream) == 0
torch.cuda.synchronize()
c1 = (ctypes.c_ulonglong * 8)()
L.sm_diag_counts(c1)
d = [c1[i] - c0[i] for i in range(8)]
nb = d[0]
print("%s: batches %d, tags/batch %.2f, in-order tags/batch %.3f (offset<16: %.3f, source before the first pending "
      "tag: %.3f), batches with a tail %.3f, 16-B passes/batch %.3f"
      % (data, nb, d[4] / nb, d[1] / nb, d[2] / nb, d[3] / nb, d[5] / nb, d[6] / nb))
