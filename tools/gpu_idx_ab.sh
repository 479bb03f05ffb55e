# Path-4 index kernel time with and without the entry lanes' walks (design tool; GPU box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/idx
for L in "" tools/var/lib_nolanes.so; do
  export SNAPPY_MI355X_LIB=$L
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/idx/v${L##*/} -o run -- python3 tools/small_prof.py html 30 > gpurun_out/idx/log 2>&1
  echo "== lib ${L:-default}"; python3 -c "
import csv,glob
f=glob.glob('gpurun_out/idx/v${L##*/}/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)): print('%-40s %5s %10.1f us' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))"
done
