# kernel trace of repeated single calls: bash tools/gpu_prof1.sh <tag> <file:op> ...
set -u
T=$1; shift
O=gpurun_out/prof1_$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 tools/single_loop.py "$@" > $O/log 2>&1 || { echo prof failed; tail $O/log; exit 1; }
python3 - $O/run_kernel_stats.csv <<'P'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print("  %-40s %5s calls %7.1f us avg  min %7.1f" % (r['Name'].split('(')[0][:40], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))
P
