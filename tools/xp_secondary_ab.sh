# Parity of the secondary kernels on the library under test, then interleaved
# A/Bs of the scrub, the encoder and the compaction against other builds:
#   bash tools/xp_secondary_ab.sh <tag> <lib-under-test> <lib> [<lib> ...]
set -o pipefail
TAG=${1:?tag}; TEST=${2:?lib}; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
GCK_LIB_PATH=$TEST timeout -k 10 600 python -u -m pytest tests/test_gpu_get.py tests/test_gpu_encode_batch.py \
  tests/test_gpu_compact.py tests/test_gpu_merge.py tests/test_gpu_hints.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
for rep in 1 2 3; do for lib in "$@"; do
  echo "scrub $lib $(GCK_LIB_PATH=$lib timeout -k 10 150 python tools/scrub.py 2>/dev/null | tail -1)"
  echo "enc $lib $(GCK_LIB_PATH=$lib timeout -k 10 120 python tools/bench_encode.py 2>/dev/null | tail -1)"
  echo "cmp $lib $(GCK_LIB_PATH=$lib timeout -k 10 150 python tools/bench_compact.py 2>/dev/null | tail -1)"
done; done | tee gpurun_out/$TAG/ab.log
