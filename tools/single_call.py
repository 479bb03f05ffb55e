"""bench.py's single-call table alone (design tool, GPU box): python tools/single_call.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package_cached()
print(json.dumps(bench.single_call_table(sm), indent=1))
