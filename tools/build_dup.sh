#!/bin/bash
# Builds SC_DUP variants of the library (design tool): tools/build_dup.sh BITS... -> tools/abl/lib_dup_<bits>.so
set -e
cd "$(dirname "$0")/.."
for b in "$@"; do
  make -s -C snappy.jl_amd/csrc -j8 SM_VARIANT=1 OUT=../../tools/abl/lib_dup_$b.so OBJ=build_dup_$b EXTRA="-DSC_DUP=$b" >/dev/null
done
