#!/bin/bash
# Builds the whole library at a git revision into tools/ablib/lib_<name>.so (design tool, for
# same-box A/B with tools/ab_raw.py): tools/build_rev.sh <name> <rev> [EXTRA flags]
set -e
cd "$(dirname "$0")/.."
T=/tmp/rev_$1
rm -rf $T && git worktree add -f $T "$2" -q
mkdir -p tools/ablib
make -s -C $T/snappy.jl_amd/csrc -j8 SM_VARIANT=1 OUT=$PWD/tools/ablib/lib_$1.so VERSION=$1 EXTRA="$3" 2>&1 | grep -v warning || true
git worktree remove --force $T
ls -la tools/ablib/lib_$1.so
