export TMPDIR=/tmp
set -e
for v in 2048 512 1024 4096; do
  lib=gocask_amd/libgocask_hip.so; [ $v != 2048 ] && lib=gocask_amd/var/libgocask_hip_lm$v.so
  GCK_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lm$v -o run -- python tools/bench_encode.py --iters 3 > gpurun_out/lm$v.json 2>/dev/null
  echo "$v $(python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_lm$v/run_kernel_stats.csv')):
    if 'k_encode_batch' in r['Name']: print(r['AverageNs'], r['MinNs'])
")"
done
