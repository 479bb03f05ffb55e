# decoder window / occupancy variants: time (ab_raw) and FETCH_SIZE (one PMC pass each)
set -u
O=gpurun_out/win; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 tools/ab_raw.py --rounds 3 tools/ablib/lib_w0.so tools/ablib/lib_w1.so tools/ablib/lib_w2.so tools/ablib/lib_w3.so > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
for l in w0 w1 w2 w3; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/p_$l -o p -- python3 tools/ab_raw.py --rounds 1 --reps 2 tools/ablib/lib_$l.so > $O/p_$l.log 2>&1 || { echo "pmc $l failed"; tail -3 $O/p_$l.log; exit 1; }
done
grep -v amdgpu.ids $O/ab.log | grep med
python3 - $O <<'P'
import csv, glob, os, sys
O = sys.argv[1]
for l in ("w0", "w1", "w2", "w3"):
    f = glob.glob(os.path.join(O, "p_" + l, "**", "*counter_collection.csv"), recursive=True)
    v = [float(r["Counter_Value"]) * 1024 for r in csv.DictReader(open(f[0])) if r["Kernel_Name"].startswith("sm::k_decompress(")]
    print(l, "k_decompress raw FETCH per launch: %.3f GB (%d launches)" % (sum(v) / len(v) / 1e9 if v else -1, len(v)))
P
