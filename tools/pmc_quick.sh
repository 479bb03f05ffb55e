#!/bin/bash
# One PMC pass (instruction counts) of the bench workload for each library given (design tool, GPU
# box): tools/pmc_quick.sh <outdir> lib.so ...   Uses tools/ab_raw.py --rounds 1 --reps 2.
set -u
O=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$O"
i=0
for L in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    -d "$O/l$i" -o p -- python3 tools/ab_raw.py --rounds 1 --reps 2 ${ABFLAGS:-} "$L" > "$O/l$i.log" 2>&1 || { echo "pmc $L failed"; tail -3 "$O/l$i.log"; exit 1; }
  echo "$L" > "$O/l$i.name"
done
python3 - "$O" <<'P'
import csv, collections, glob, os, sys
O = sys.argv[1]
for d in sorted(glob.glob(os.path.join(O, "l*"))):
    if not os.path.isdir(d):
        continue
    name = open(d + ".name").read().strip()
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "k_compress_sc" not in k and "k_decompress" not in k:
            continue
        k = "compress" if "k_compress_sc" in k else "decompress"
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES":
            n[k] += 1
    for k, v in agg.items():
        print("%-40s %-10s" % (os.path.basename(name), k), " ".join("%s=%.3f" % (c[9:], x / n[k] / 655.36e6) for c, x in sorted(v.items()) if c != "SQ_WAVES"))
P
