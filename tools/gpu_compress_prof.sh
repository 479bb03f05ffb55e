# Kernel traces of single sm_compress calls on the reference's benchmark files (design tool; GPU box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cprof
for f in html fireworks.jpeg paper-100k.pdf sample-tweet.json; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cprof/$f -o run -- python3 tools/compress_prof.py $f 30 > gpurun_out/cprof/$f.log 2>&1 || { echo prof failed; tail gpurun_out/cprof/$f.log; exit 1; }
  echo "== $f"; python3 -c "
import csv,glob
f=glob.glob('gpurun_out/cprof/$f/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)): print('%-40s %5s %10.1f us' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))"
done
