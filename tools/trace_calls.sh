# rocprofv3 kernel traces of single-call uncompress for the named corpus files, one summary line
# per kernel (design tool, GPU box): bash tools/trace_calls.sh html paper-100k.pdf ...
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for f in "$@"; do
  rm -rf gpurun_out/st_$f
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_$f -o st -- python3 tools/single_trace.py $f > /dev/null || exit 1
  python3 - gpurun_out/st_$f $f <<'P'
import csv, glob, sys
g = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
rows = [r for r in csv.DictReader(open(g[0])) if int(r["Calls"]) >= 50]
print(sys.argv[2], " ".join("%s=%.1f" % (r["Name"].split("(")[0].split("::")[-1].split("<")[0], float(r["AverageNs"]) * int(r["Calls"]) / 50e3) for r in rows))
P
done
