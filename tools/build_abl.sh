#!/bin/bash
# Builds ablation variants of the library (design tool): tools/build_abl.sh BITS... -> tools/abl/lib_abl_<bits>.so
set -e
cd "$(dirname "$0")/.."
for b in "$@"; do
  make -s -C snappy.jl_amd/csrc -j8 OUT=../../tools/abl/lib_abl_$b.so OBJ=build_abl_$b EXTRA="-DSC_ABL=$b" >/dev/null
done
