set -u
O=gpurun_out/mask2; rm -rf $O; mkdir -p $O
for l in s0 s2; do
  echo "== m0 vs $l" >> $O/log.txt
  timeout -k 10 400 python3 tools/ab_bytes.py tools/ablib/lib_m0.so tools/ablib/lib_$l.so >> $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
done
timeout -k 10 300 python3 tools/ab_raw.py --rounds 3 --compress-only tools/ablib/lib_m0.so tools/ablib/lib_m1.so tools/ablib/lib_s0.so tools/ablib/lib_s2.so > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
timeout -k 10 300 python3 tools/ab_raw.py --rounds 3 --compress-only --data large tools/ablib/lib_m0.so tools/ablib/lib_m1.so tools/ablib/lib_s0.so tools/ablib/lib_s2.so > $O/abl.log 2>&1 || { tail $O/abl.log; exit 1; }
grep -v amdgpu.ids $O/log.txt | grep -E "==|text|config|geo|small|SAME|DIFF"; grep -v amdgpu.ids $O/ab.log | grep med; grep -v amdgpu.ids $O/abl.log | grep med
