"""Fast-mode stream size per corpus file against the reference's (the oracle, reference mode):
python tools/fast_sizes.py  (GPU box; design/report tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench  # noqa: E402
import oracle as O  # noqa: E402


def main():
    sm = bench.load_package()
    tdir = os.path.join(ROOT, "tests", "golden", "testdata")
    worst = worstd = 0.0
    for f in sorted(os.listdir(tdir)):
        if f.endswith(".snappy") or f.startswith("baddata"):
            continue
        raw = open(os.path.join(tdir, f), "rb").read()
        ref = len(O.compress(raw))
        fast = sm.compress(raw, mode="fast")
        dense = sm.compress(raw, mode="dense")
        assert O.uncompress(fast) == raw and O.uncompress(dense) == raw
        r, rd = len(fast) / ref, len(dense) / ref
        worst = max(worst, r)
        worstd = max(worstd, rd)
        print("%-20s %9d  ref %9d  fast %9d (%.4f)  dense %9d (%.4f)" % (f, len(raw), ref, len(fast), r, len(dense), rd))
    print("worst fast/ref %.4f, dense/ref %.4f" % (worst, worstd))


if __name__ == "__main__":
    main()
