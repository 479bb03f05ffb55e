# round-3 session: decoder ablations/stamps, occupancy A/B, compressor stamps (design measurements)
set -u
bash tools/gpu_dec.sh s3c || exit 1
OP=uncompress bash tools/gpu_ab.sh s3c_occ tools/abl/lib_occ8.so tools/abl/lib_occ6.so || exit 1
bash tools/gpu_stamps.sh s3c
