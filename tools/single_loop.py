"""Repeated single calls of one file for a kernel trace (design tool, GPU box):
python3 tools/single_loop.py <file>:<u|c> ... (200 calls each)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package_cached()
for spec in sys.argv[1:]:
    f, op = spec.split(":")
    data = open(os.path.join(ROOT, "tests", "golden", "testdata", f), "rb").read()
    comp = sm.compress(data, mode="fast")
    for _ in range(200):
        sm.uncompress(comp) if op == "u" else sm.compress(data, mode="fast")
