#!/bin/bash
# Build the product library of another revision for interleaved A/Bs:
#   bash tools/build_rev.sh <git rev> <name>   -> gocask_amd/var/libgocask_hip_<name>.so
set -e
rev=$1; name=$2
d=$(mktemp -d /tmp/gck_rev_XXXX)
git archive "$rev" gocask_amd/csrc include | tar -x -C "$d"
make -s -j8 -C "$d/gocask_amd/csrc" OUT="$PWD/gocask_amd/var/libgocask_hip_$name.so" BUILD=build \
  "$PWD/gocask_amd/var/libgocask_hip_$name.so" 2>&1 | grep -v warning || true
rm -rf "$d"
ls -la gocask_amd/var/libgocask_hip_$name.so
