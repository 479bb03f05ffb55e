"""Same-box A/B of library builds on the bench workload (design tool; run on the GPU box).

  python tools/ab_raw.py [--blocks 10000] [--reps 20] [--rounds 3] [--data text|random] lib.so ...

Loads each build with only the batch entry points (sm_ctx_create, sm_compress_batch_device,
sm_uncompress_batch_device), so builds from older commits with other symbol sets compare too.
Per build and round: fast-mode compress and uncompress of the same device-resident blocks,
median of `reps` launches from HIP events on the launch stream; the builds alternate within a
round, so box drift hits all of them alike.  Every build's streams must decode bit-exactly
(through its own decoder) or the script exits 1.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    L.sm_ctx_create.restype = vp
    L.sm_ctx_create.argtypes = [ctypes.c_int]
    L.sm_compress_batch_device.restype = ctypes.c_int32
    L.sm_compress_batch_device.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, ctypes.c_int, vp]
    L.sm_uncompress_batch_device.restype = ctypes.c_int32
    L.sm_uncompress_batch_device.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, vp, vp, vp]
    return L, L.sm_ctx_create(0)


def p(t):
    return ctypes.c_void_p(t.data_ptr())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--data", default="text")
    ap.add_argument("--mode", type=int, default=1)  # SM_MODE_FAST
    ap.add_argument("--no-verify", action="store_true", help="ablation builds: their streams are not valid")
    ap.add_argument("--compress-only", action="store_true")
    ap.add_argument("--decode-ablation", action="store_true",
                    help="the first build compresses once; every build's uncompress of those streams is timed, "
                         "unverified (decoder ablation builds)")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if a.data == "large":  # config 5's corpus cut into its 10,304 64 KiB fragments, as a batch of blocks
        blocks = bench.large_corpus().reshape(-1, bench.BLOCK)
    else:
        blocks = bench.text_blocks(a.blocks, 0x5EED) if a.data == "text" else bench.random_blocks(a.blocks, 0x5EED + 1)
    B = bench.Batch(blocks, dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    libs = [(os.path.basename(x), *load(x)) for x in a.libs]

    def comp(L, ctx):
        st = L.sm_compress_batch_device(ctx, p(B.d_in), p(B.in_off), p(B.in_len), B.nblk, p(B.d_comp), p(B.comp_off),
                                        p(B.comp_len), a.mode, stream)
        assert st == 0, st

    def unc(L, ctx):
        st = L.sm_uncompress_batch_device(ctx, p(B.d_comp), p(B.comp_off), p(B.comp_len), B.nblk, p(B.d_dec),
                                          p(B.in_off), p(B.dec_cap), p(B.dec_len), p(B.status), stream)
        assert st == 0, st

    res = {name: {"c": [], "u": []} for name, _, _ in libs}
    if a.decode_ablation:
        comp(libs[0][1], libs[0][2])
        torch.cuda.synchronize()
        for r in range(a.rounds):
            for name, L, ctx in libs:
                um = bench.kernel_ms(lambda: unc(L, ctx), a.reps)
                res[name]["u"].append(um)
                print("round %d %-28s uncompress %.4f ms" % (r, name, um), flush=True)
        for name, v in res.items():
            print("%-28s uncompress min %.4f med %.4f" % (name, min(v["u"]), float(np.median(v["u"]))))
        return
    ok = True
    for r in range(a.rounds):
        for name, L, ctx in libs:
            comp(L, ctx)
            torch.cuda.synchronize()
            ratio = float(B.comp_len.to(torch.int64).sum()) / B.in_bytes
            good = False
            if not a.no_verify:  # (an ablation's slots hold no valid streams: not decoded at all)
                B.d_dec.fill_(0xAA)
                unc(L, ctx)
                torch.cuda.synchronize()
                good = bool(torch.equal(B.d_dec, B.d_in)) and int(B.status.abs().sum()) == 0
                ok &= good
            cm = bench.kernel_ms(lambda: comp(L, ctx), a.reps)
            um = 0.0 if (a.compress_only or a.no_verify) else bench.kernel_ms(lambda: unc(L, ctx), a.reps)
            res[name]["c"].append(cm)
            res[name]["u"].append(um)
            print("round %d %-28s compress %.4f ms  uncompress %.4f ms  ratio %.4f  roundtrip %s"
                  % (r, name, cm, um, ratio, "ok" if good else "FAILED"), flush=True)
    for name, v in res.items():
        print("%-28s compress min %.4f med %.4f | uncompress min %.4f med %.4f" % (
            name, min(v["c"]), float(np.median(v["c"])), min(v["u"]), float(np.median(v["u"]))))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
