set -o pipefail
out=gpurun_out/r4zzd
mkdir -p $out
L=gocask_amd/var
for v in gs8 gs4; do
  GCK_LIB_PATH=$L/libgocask_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_get.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest_$v.log 2>&1 || { tail -5 $out/pytest_$v.log; exit 1; }
  tail -1 $out/pytest_$v.log
done
for rep in 1 2; do for lib in head gs8 gs4; do
  echo "$lib $(GCK_LIB_PATH=$L/libgocask_hip_$lib.so timeout -k 10 300 python tools/bench_get.py 2>&1 | tail -1)" >> $out/get_ab.log || exit 1
done; done
cat $out/get_ab.log
