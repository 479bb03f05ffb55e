"""Summarise rocprofv3 --pmc CSV passes: per kernel, the mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict


def summarise(root, kernel_filter=None):
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "?")
            if kernel_filter and kernel_filter not in k:
                continue
            name = row["Counter_Name"]
            vals[k][(name, row.get("Dispatch_Id"))].append(float(row["Counter_Value"]))
    out = {}
    for k, d in vals.items():
        per = defaultdict(list)
        for (name, _), v in d.items():
            per[name].append(sum(v))
        out[k] = {n: sum(v) / len(v) for n, v in per.items()}
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
    for k, d in res.items():
        print(k[:80])
        for n in sorted(d):
            print("   %-24s %16.1f" % (n, d[n]))
