set -o pipefail
out=gpurun_out/r4zzh
mkdir -p $out
L=gocask_amd/var
for rep in 1 2; do for lib in cw16 cw12 cw20 cw24; do
  echo "$lib $(GCK_LIB_PATH=$L/libgocask_hip_$lib.so timeout -k 10 300 python tools/bench_compact.py 2>&1 | tail -1)" >> $out/cmp_ab.log || exit 1
done; done
cut -c1-220 $out/cmp_ab.log
