#!/bin/bash
# Builds a named variant of the library (design tool): tools/build_var.sh NAME "EXTRA flags" -> tools/abl/lib_NAME.so
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/abl
make -s -C snappy.jl_amd/csrc -j8 SM_VARIANT=1 OUT=../../tools/abl/lib_$1.so OBJ=build_var_$1 EXTRA="$2" >/dev/null
