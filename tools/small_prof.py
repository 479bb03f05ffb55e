"""Path-4 single calls for a kernel trace (design tool, GPU box):
rocprofv3 --kernel-trace --stats -d gpurun_out/x -- python3 tools/small_prof.py [file] [calls]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package_cached()
f = sys.argv[1] if len(sys.argv) > 1 else "html"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
raw = open(os.path.join(ROOT, "tests", "golden", "testdata", f), "rb").read()
comp = sm.compress(raw)
for _ in range(n):
    assert sm.uncompress(comp) == raw
print(f, "path", sm.last_uncompress_path())
