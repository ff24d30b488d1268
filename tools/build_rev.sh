#!/bin/bash
# Build the product library of another revision for interleaved A/Bs:
#   bash tools/build_rev.sh <git rev> <name>   -> gocask_amd/var/libgocask_hip_<name>.so
set -e
rev=$1; name=$2
d=$(mktemp -d /tmp/gck_rev_XXXX)
git archive "$rev" gocask_amd/csrc include | tar -x -C "$d"
# this tree's Makefile (its diag rule links the variant library by path)
cp gocask_amd/csrc/Makefile "$d/gocask_amd/csrc/Makefile"
# (and its own diag library: diag.hip reads the context's layout)
make -s -j8 -C "$d/gocask_amd/csrc" OUT="$PWD/gocask_amd/var/libgocask_hip_$name.so" BUILD=build \
  DIAG="$PWD/gocask_amd/var/libgocask_diag_$name.so" all 2>&1 | grep -v warning || true
rm -rf "$d"
ls -la gocask_amd/var/libgocask_hip_$name.so
