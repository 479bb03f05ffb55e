"""Single sm_compress calls for a kernel trace (design tool, GPU box):
rocprofv3 --kernel-trace --stats -d gpurun_out/x -- python3 tools/compress_prof.py [file] [calls] [mode]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package_cached()
f = sys.argv[1] if len(sys.argv) > 1 else "html"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
mode = sys.argv[3] if len(sys.argv) > 3 else "fast"
raw = open(os.path.join(ROOT, "tests", "golden", "testdata", f), "rb").read()
for _ in range(n):
    c = sm.compress(raw, mode=mode)
assert sm.uncompress(c) == raw
print(f, len(raw), "->", len(c))
