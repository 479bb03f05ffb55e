"""One file's single-call uncompress (and compress) repeated, for a rocprofv3 kernel trace of the
single-call paths (design tool, GPU box):
  rocprofv3 --kernel-trace --stats -d gpurun_out/st -o st -- python3 tools/single_trace.py html"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package_cached()
f = sys.argv[1] if len(sys.argv) > 1 else "html"
data = open(os.path.join(ROOT, "tests", "golden", "testdata", f), "rb").read()
comp = sm.compress(data, mode="fast")
for _ in range(50):
    assert sm.uncompress(comp) == data
print(f, "path", sm.last_uncompress_path())
