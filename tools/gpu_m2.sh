set -u
O=gpurun_out/m2; rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 tools/ab_bytes.py tools/ablib/lib_m1n.so tools/ablib/lib_m2.so > $O/bytes.txt 2>&1 || { tail $O/bytes.txt; exit 1; }
timeout -k 10 300 python3 tools/ab_raw.py --rounds 3 --compress-only tools/ablib/lib_m1n.so tools/ablib/lib_m2.so > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
timeout -k 10 300 python3 tools/ab_raw.py --rounds 3 --compress-only --data large tools/ablib/lib_m1n.so tools/ablib/lib_m2.so > $O/abl.log 2>&1 || { tail $O/abl.log; exit 1; }
grep -v amdgpu.ids $O/bytes.txt | tail -3; grep med $O/ab.log; grep med $O/abl.log
