set -o pipefail
out=gpurun_out/r4zzc
mkdir -p $out
L=gocask_amd/var
GCK_LIB_PATH=$L/libgocask_hip_gs16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_get.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { tail -5 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
bash tools/scrub_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_gs16.so > $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
bash tools/scrub_ab.sh $L/libgocask_hip_head.so $L/libgocask_hip_gs16.so >> $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
cat $out/scrub_ab.log
for rep in 1 2; do for lib in head gs16; do
  echo "$lib $(GCK_LIB_PATH=$L/libgocask_hip_$lib.so timeout -k 10 300 python tools/bench_get.py 2>&1 | tail -1)" >> $out/get_ab.log || exit 1
done; done
cat $out/get_ab.log
