set -o pipefail
out=gpurun_out/r4zzj
mkdir -p $out
L=gocask_amd/var
GCK_LIB_PATH=$L/libgocask_hip_ctop.so timeout -k 10 400 python -u -m pytest tests/test_gpu_compact.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -15 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do for lib in head ctop; do
  echo "$lib $(GCK_LIB_PATH=$L/libgocask_hip_$lib.so timeout -k 10 300 python tools/bench_compact.py 2>&1 | tail -1)" >> $out/cmp_ab.log || exit 1
done; done
cut -c1-200 $out/cmp_ab.log
