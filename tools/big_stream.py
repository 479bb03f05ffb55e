"""Single-stream (whole-buffer API) timing on a large input (design tool, GPU box):
sm_compress / sm_uncompress of one snappy stream of --mb MiB (the corpus tiled), host buffers.

  python3 tools/big_stream.py --mb 64
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    sm = bench.load_package()
    corpus = b"".join(open(os.path.join(bench.TESTDATA, f), "rb").read() for f in bench.TEXTS)
    n = args.mb << 20
    raw = (corpus * (n // len(corpus) + 1))[:n]
    for mode in ("fast", "reference"):
        comp = sm.compress(raw, mode=mode)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            comp = sm.compress(raw, mode=mode)
        tc = (time.perf_counter() - t0) / args.reps
        back = sm.uncompress(comp)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            back = sm.uncompress(comp)
        td = (time.perf_counter() - t0) / args.reps
        print("%s: %d MiB -> %.3f ratio; compress %.2f GB/s, uncompress %.2f GB/s (host buffers, incl. PCIe); "
              "ok %s; decode path %d" % (mode, args.mb, len(comp) / n, n / tc / 1e9, n / td / 1e9, back == raw,
                                         sm.last_uncompress_path()))


if __name__ == "__main__":
    main()
