"""Fast- and dense-mode streams of the corpus files, written to gpurun_out/streams/ (design tool,
GPU box): CPU models of the decoders' path structure read them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sm = bench.load_package_cached()
td = os.path.join(ROOT, "tests", "golden", "testdata")
od = os.path.join(ROOT, "gpurun_out", "streams")
os.makedirs(od, exist_ok=True)
for f in sorted(os.listdir(td)):
    if f.endswith(".snappy") or f.startswith("baddata"):
        continue
    raw = open(os.path.join(td, f), "rb").read()
    for mode in ("fast", "dense"):
        c = sm.compress(raw, mode=mode)
        assert sm.uncompress(c) == raw
        open(os.path.join(od, "%s.%s" % (f, mode)), "wb").write(c)
print("dumped", len(os.listdir(od)))
