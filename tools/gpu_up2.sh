set -u
O=gpurun_out/up2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for spec in fireworks.jpeg:u sample-tweet.json:u sample-tweet.json:c; do
  n=${spec//[:.]/_}
  SNAPPY_MI355X_LIB=tools/ablib/lib_up2.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 tools/single_loop.py $spec > $O/$n.log 2>&1 || { echo prof failed; tail $O/$n.log; exit 1; }
done
for f in $(find $O -name "*kernel_stats.csv"); do echo "== $f"; cut -d, -f1-8 $f | head -12; done
