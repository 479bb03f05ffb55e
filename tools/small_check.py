"""Path 4 (small streams decoded on the device) against the oracle (design check, GPU box):
corpus files in every compress mode, built streams that stress the origin pointers, mutated
streams (status parity), and per-call times with path 4 on and off.  python tools/small_check.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench  # noqa: E402
import oracle as O  # noqa: E402
from streams import build, random_ops  # noqa: E402


def status(sm, fn, s):
    try:
        return 0, fn(s)
    except sm.SnappyError as e:
        return e.code, None


def main():
    sm = bench.load_package_cached()
    td = os.path.join(ROOT, "tests", "golden", "testdata")
    files = sorted(f for f in os.listdir(td) if not f.endswith(".snappy"))
    bad = 0
    paths = {}
    for f in files:
        raw = open(os.path.join(td, f), "rb").read()
        for name, comp in (("oracle", O.compress(raw)), ("fast", sm.compress(raw)), ("dense", sm.compress(raw, mode="dense"))):
            got = sm.uncompress(comp)
            p = sm.last_uncompress_path()
            paths[p] = paths.get(p, 0) + 1
            if got != raw:
                bad += 1
                print("MISMATCH", f, name, p)
    rng = np.random.default_rng(5)
    cases = [build([("lit", b"x")] + [("copy", 1, 64)] * 3000), build(random_ops(rng, 200_000)),
             build(random_ops(rng, 50_000, long_lit_p=0.2)), build(random_ops(rng, 900_000, near=60_000))]
    ops, size = [("lit", rng.integers(0, 256, 5000, dtype=np.uint8).tobytes())], 5000
    for _ in range(3000):
        ln = int(rng.integers(4, 65))
        ops.append(("copy", size, ln))
        size += ln
    cases.append(build(ops))
    for i, (s, e) in enumerate(cases):
        got = sm.uncompress(s)
        p = sm.last_uncompress_path()
        paths[p] = paths.get(p, 0) + 1
        if got != e:
            bad += 1
            print("MISMATCH built", i, p)
    # mutations: the status (and output when valid) equals the oracle's
    nm = 0
    for f in ("html", "alice29.txt", "urls.10K", "fireworks.jpeg", "sample-tweet.json"):
        good = sm.compress(open(os.path.join(td, f), "rb").read())
        for _ in range(40):
            b = bytearray(good)
            for _ in range(int(rng.integers(1, 4))):
                b[int(rng.integers(3, len(b)))] = int(rng.integers(0, 256))
            b = bytes(b)
            st_o, out_o = O.uncompress_status(b) if hasattr(O, "uncompress_status") else (None, None)
            st_g, out_g = status(sm, sm.uncompress, b)
            nm += 1
            if st_g != st_o or (st_o == 0 and out_g != out_o):
                bad += 1
                print("MUTATION MISMATCH", f, st_g, st_o)
    print("paths", paths, "mutations", nm, "mismatches", bad)
    for f in ("sample-tweet.json", "html", "alice29.txt", "urls.10K", "fireworks.jpeg", "paper-100k.pdf"):
        raw = open(os.path.join(td, f), "rb").read()
        comp = sm.compress(raw)
        row = []
        for on in (1, 0):
            sm.set_small_decode(on)
            sm.uncompress(comp)
            ts = []
            for _ in range(30):
                t0 = time.perf_counter()
                sm.uncompress(comp)
                ts.append(time.perf_counter() - t0)
            t = float(np.median(ts))
            row.append("path %d %7.1f us (%6.1f MB/s compressed)" % (sm.last_uncompress_path(), t * 1e6, len(comp) / t / 2**20))
        sm.set_small_decode(1)
        print("%-18s %7d -> %7d: %s" % (f, len(raw), len(comp), " | ".join(row)))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
