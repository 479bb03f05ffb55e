# Path-4 kernel traces of single uncompress calls (html, paper-100k.pdf) + tools/small_check.py
# (design tool; GPU box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/small_prof
for f in html paper-100k.pdf; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/small_prof/$f -o run -- python3 tools/small_prof.py $f 30 > gpurun_out/small_prof/$f.log 2>&1 || { echo prof failed; tail gpurun_out/small_prof/$f.log; exit 1; }
  echo "== $f"; python3 -c "
import csv,glob
f=glob.glob('gpurun_out/small_prof/$f/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)): print('%-40s %5s %10.1f us' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))"
done
timeout -k 10 200 python3 tools/small_check.py > gpurun_out/small_prof/small.log 2>&1; echo "small rc $?"; tail -8 gpurun_out/small_prof/small.log
