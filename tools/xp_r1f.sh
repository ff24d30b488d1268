# Round-1 re-entry check + fused-pass ablation (k_fuse with and without the
# header-chain parse): bash tools/xp_r1f.sh
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest ok"
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --verbose > gpurun_out/bench_default.log 2>&1
echo "bench default ok"
for v in base noparse; do
  lib=gocask_amd/libgocask_hip.so
  [ $v = noparse ] && lib=gocask_amd/var/libgocask_hip_noparse.so
  GCK_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$v -o run -- python bench.py --fused --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/fused_$v.log 2>&1
  echo "fused $v ok"
done
