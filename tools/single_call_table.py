"""The INTEGRATION.md single-call table from a bench.py --extras JSON line (design tool):
python3 tools/single_call_table.py profiles/r04_bench.json"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
files = d["single_call"]["files"]
print("| file | compress MB/s fast / dense (reference) | uncompress MB/s fast (reference) | us: compress fast, uncompress fast |")
print("|---|---|---|---|")
for tag in ("txt", "html", "urls", "jpeg", "pdf", "json"):
    r = files[tag]
    j = r["julia_published_MBps"]
    print("| %s | %s / %s (%s) | %s (%s) | %s, %s |" % (
        r["file"], format(r["fast"]["compress_MBps"], ",.0f"), format(r["dense"]["compress_MBps"], ",.0f"),
        format(j["compress"], ",.0f"), format(r["fast"]["uncompress_MBps"], ",.0f"), format(j["uncompress"], ",.0f"),
        r["fast"]["compress_us"], r["fast"]["uncompress_us"]))
