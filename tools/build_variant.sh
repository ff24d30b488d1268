# Build a variant of the product library from a sed-edited copy of csrc:
#   bash tools/build_variant.sh <name> <file.hip> '<sed expr>' [more file/expr pairs]
#   -> gocask_amd/var/libgocask_hip_<name>.so
set -e
name=$1; shift
d=gocask_amd/csrc_x_$name
rm -rf $d && mkdir -p $d && cp gocask_amd/csrc/*.hip gocask_amd/csrc/*.h gocask_amd/csrc/*.cpp gocask_amd/csrc/Makefile $d/
while [ $# -ge 2 ]; do
  f=$1; expr=$2; shift 2
  sed -i "$expr" $d/$f
  if cmp -s $d/$f gocask_amd/csrc/$f; then echo "sed changed nothing in $f" >&2; exit 1; fi
done
make -s -j8 -C $d OUT=../var/libgocask_hip_$name.so DIAG=../var/libgocask_diag_$name.so BUILD=build all 2>&1 | grep -v warning || true
ls -la gocask_amd/var/libgocask_hip_$name.so
