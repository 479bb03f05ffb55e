# Ablation, stamp and PMC runs of the fast compressor (design measurements; run on the GPU box)
set -u
O=gpurun_out/${1:-abl}
mkdir -p $O
timeout -k 10 120 python3 tools/sc_abl.py --label base > $O/abl.log 2>&1 || { echo base failed; tail $O/abl.log; exit 1; }
for L in tools/abl/lib_abl_*.so; do
  SNAPPY_MI355X_LIB=$L timeout -k 10 120 python3 tools/sc_abl.py >> $O/abl.log 2>&1 || { echo "$L failed"; tail $O/abl.log; exit 1; }
done
cat $O/abl.log
if [ -f tools/abl/lib_stamp.so ]; then
  SNAPPY_MI355X_LIB=tools/abl/lib_stamp.so timeout -k 10 120 python3 tools/sc_stamps.py > $O/stamps.log 2>&1 || { echo stamps failed; tail $O/stamps.log; exit 1; }
  cat $O/stamps.log
fi
if [ "${PMC:-1}" = 1 ]; then
  BLOCKS=10000 bash tools/pmc_run.sh compress_fast $O/pmc_compress text > $O/pmc.log 2>&1 || { echo pmc failed; tail $O/pmc.log; exit 1; }
  python3 tools/pmc_summary.py $O/pmc_compress k_compress_sc
fi
echo done
