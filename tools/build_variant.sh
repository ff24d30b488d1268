# Build a variant of the product library from a sed-edited copy of csrc:
#   bash tools/build_variant.sh <name> '<sed expr on replay.hip>' [extra make args]
#   -> gocask_amd/var/libgocask_hip_<name>.so
set -e
name=$1; expr=$2; shift 2
d=gocask_amd/csrc_x_$name
rm -rf $d && mkdir -p $d && cp gocask_amd/csrc/*.hip gocask_amd/csrc/*.h gocask_amd/csrc/*.cpp gocask_amd/csrc/Makefile $d/
sed -i "$expr" $d/replay.hip
if cmp -s $d/replay.hip gocask_amd/csrc/replay.hip; then echo "sed changed nothing" >&2; exit 1; fi
make -s -j8 -C $d OUT=../var/libgocask_hip_$name.so DIAG=/dev/null/x BUILD=build "$@" ../var/libgocask_hip_$name.so 2>&1 | grep -v warning || true
ls -la gocask_amd/var/libgocask_hip_$name.so
