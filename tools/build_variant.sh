#!/bin/bash
# Builds the library with one source file replaced (design tool): tools/build_variant.sh <name> <file.hip> <replacement>
# -> tools/ablib/lib_<name>.so (travels to the GPU box)
set -e
cd "$(dirname "$0")/.."
T=/tmp/variant_$1
rm -rf $T && mkdir -p $T/snappy.jl_amd $T/include
cp -r snappy.jl_amd/csrc $T/snappy.jl_amd/ && rm -rf $T/snappy.jl_amd/csrc/build*
cp include/*.h $T/include/
cp "$3" $T/snappy.jl_amd/csrc/$2
mkdir -p tools/ablib
make -s -C $T/snappy.jl_amd/csrc -j8 SM_VARIANT=1 OUT=$PWD/tools/ablib/lib_$1.so VERSION=$1 2>&1 | grep -v warning || true
ls -la tools/ablib/lib_$1.so
