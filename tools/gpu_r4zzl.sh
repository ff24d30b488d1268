set -o pipefail
out=gpurun_out/r4zzl
mkdir -p $out
L=gocask_amd/var
GCK_LIB_PATH=$L/libgocask_hip_kd16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_merge.py tests/test_gpu_get.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -15 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do for lib in head kd2 kd4 kd16; do
  echo "$lib $(GCK_LIB_PATH=$L/libgocask_hip_$lib.so timeout -k 10 300 python tools/kd_time.py 2>&1 | tail -2 | tr '\n' ' ')" >> $out/kd_ab.log || exit 1
done; done
cat $out/kd_ab.log
