#!/bin/bash
# Builds the library with one source file replaced (design tool): tools/build_variant.sh <name> <file.hip> <replacement>
# -> tools/abl/lib_<name>.so
set -e
cd "$(dirname "$0")/.."
T=/tmp/variant_$1
rm -rf $T && mkdir -p $T/snappy.jl_amd $T/include
cp -r snappy.jl_amd/csrc $T/snappy.jl_amd/ && rm -rf $T/snappy.jl_amd/csrc/build*
cp include/*.h $T/include/
cp "$3" $T/snappy.jl_amd/csrc/$2
mkdir -p tools/abl
make -s -C $T/snappy.jl_amd/csrc -j8 OUT=$PWD/tools/abl/lib_$1.so VERSION=$1 2>&1 | grep -v warning || true
ls -la tools/abl/lib_$1.so
