set -u
O=gpurun_out/r06_single
mkdir -p $O
timeout -k 10 200 python3 tools/single_call.py > $O/single.json 2> $O/single.err || { echo single failed; tail $O/single.err; exit 1; }
timeout -k 10 200 python3 tools/single_phase.py fireworks.jpeg:u paper-100k.pdf:u sample-tweet.json:u sample-tweet.json:c fireworks.jpeg:c alice29.txt:c/reference html:c/reference > $O/phase.log 2>&1 || { echo phase failed; tail $O/phase.log; exit 1; }
python3 - <<'P'
import json
d=json.load(open('gpurun_out/r06_single/single.json'))
for k,v in d['files'].items():
  print(k, v['bytes'], {m:(v[m]['compressed_bytes'],v[m]['compress_us'],v[m]['uncompress_us'],v[m]['uncompress_path']) for m in ('fast','dense','reference')})
P
grep -v amdgpu.ids $O/phase.log
