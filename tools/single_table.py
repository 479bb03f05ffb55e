"""INTEGRATION.md's single-call table from a bench --extras line (design tool):
python3 tools/single_table.py profiles/r06_bench_extras.json"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("| file | compress MB/s fast / dense (reference) | uncompress MB/s fast (reference) | us: compress fast, uncompress fast (path) |")
print("|---|---|---|---|")
for k, v in d["single_call"]["files"].items():
    f, de, j = v["fast"], v["dense"], v["julia_published_MBps"]
    print("| %s | %s / %s (%s) | %s (%s) | %.1f, %.1f (%d) |" % (
        v["file"], format(round(f["compress_MBps"]), ","), format(round(de["compress_MBps"]), ","),
        format(round(j["compress"]), ","), format(round(f["uncompress_MBps"]), ","), format(round(j["uncompress"]), ","),
        f["compress_us"], f["uncompress_us"], f["uncompress_path"]))
