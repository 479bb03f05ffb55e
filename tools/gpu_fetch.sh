set -u
O=gpurun_out/fetch; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O -o p -- tools/probes/fetch_calib > $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
grep -v "^W20\|amdgpu.ids" $O/log.txt | tail -5
f=$(find $O -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'P'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r.get("Kernel_Name", r.get("Kernel-Name",""))[:40], r.get("Counter_Name"), r.get("Counter_Value"))
P
