set -u
O=gpurun_out/mask; mkdir -p $O
for l in m1 mf1 mf2; do
  echo "== m0 vs $l" >> $O/log.txt
  timeout -k 10 400 python3 tools/ab_bytes.py tools/ablib/lib_m0.so tools/ablib/lib_$l.so >> $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
done
timeout -k 10 300 python3 tools/ab_raw.py --rounds 3 --compress-only tools/ablib/lib_m0.so tools/ablib/lib_m1.so tools/ablib/lib_mf1.so tools/ablib/lib_mf2.so > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/log.txt; grep -v amdgpu.ids $O/ab.log | grep med
