#!/bin/bash
# Parity subset on one library, then an interleaved A/B of several (one GPU call):
#   bash tools/xp_ab.sh <tag> <reps> <lib-under-test> <lib> [<lib> ...]
set -o pipefail
TAG=${1:?tag}; REPS=${2:?reps}; TEST=${3:?lib}; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
D=${TEST/libgocask_hip/libgocask_diag}
GCK_LIB_PATH=$TEST GCK_DIAG_PATH=$D timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py \
  tests/test_gpu_configs.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 \
  || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
bash tools/ab_mix.sh $REPS "$@" > gpurun_out/$TAG/ab.log 2>&1 || { cat gpurun_out/$TAG/ab.log; exit 1; }
cat gpurun_out/$TAG/ab.log
