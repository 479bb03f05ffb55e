"""Same bytes from two library builds (design tool, GPU box): python3 tools/ab_bytes.py a.so b.so
Compresses the bench text, config 5's fragments and windows of each corpus file with both builds
(fast and dense modes) and compares the compressed blocks byte for byte, then times each set."""
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

libs = [load(x) for x in sys.argv[1:3]]
dev = torch.device("cuda", 0)
stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
sets = [("bench text", bench.text_blocks(2000, 0x5EED)), ("config 5", bench.large_corpus().reshape(-1, bench.BLOCK))]
for f in ("html", "kppkn.gtb", "geo.protodata", "urls.10K", "paper-100k.pdf", "smallrandom1.bin"):
    raw = np.frombuffer(open(os.path.join(bench.TESTDATA, f), "rb").read(), np.uint8)
    tiled = np.tile(raw, (2 * bench.BLOCK) // raw.size + 2)
    offs = np.random.default_rng(7).integers(0, tiled.size - bench.BLOCK, 2000)
    sets.append((f, np.ascontiguousarray(np.lib.stride_tricks.sliding_window_view(tiled, bench.BLOCK)[offs])))
ok = True
for name, blocks in sets:
    B = bench.Batch(blocks, dev)
    res = []
    for mode in (1, 2):
        outs, times = [], []
        for L, ctx in libs:
            def comp():
                assert L.sm_compress_batch_device(ctx, p(B.d_in), p(B.in_off), p(B.in_len), B.nblk, p(B.d_comp),
                                                  p(B.comp_off), p(B.comp_len), mode, stream) == 0
            comp()
            torch.cuda.synchronize()
            outs.append((B.comp_len.clone(), B.d_comp.clone()))
            times.append(bench.kernel_ms(comp, 10) if mode == 1 else 0.0)
        same = torch.equal(outs[0][0], outs[1][0])
        if same:
            lens = outs[0][0].to(torch.int64).cpu().numpy()
            offs = B.comp_off.cpu().numpy()
            a, b = outs[0][1], outs[1][1]
            for i in range(B.nblk):
                if not torch.equal(a[offs[i]:offs[i] + lens[i]], b[offs[i]:offs[i] + lens[i]]):
                    same = False
                    break
        ok &= same
        res.append("mode %d %s%s" % (mode, "same bytes" if same else "DIFFERENT", (" %.4f / %.4f ms" % tuple(times)) if mode == 1 else ""))
    print("%-18s %s" % (name, "; ".join(res)), flush=True)
print("ALL SAME" if ok else "DIFFERENCES")
sys.exit(0 if ok else 1)
