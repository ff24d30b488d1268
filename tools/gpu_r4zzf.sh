set -o pipefail
out=gpurun_out/r4zzf
mkdir -p $out
L=gocask_amd/var
GCK_LIB_PATH=$L/libgocask_hip_cmph.so timeout -k 10 400 python -u -m pytest tests/test_gpu_compact.py tests/test_oracle_compact.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -15 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do for lib in head cmph; do
  echo "$lib $(GCK_LIB_PATH=$L/libgocask_hip_$lib.so timeout -k 10 300 python tools/bench_compact.py 2>&1 | tail -1)" >> $out/cmp_ab.log || exit 1
done; done
cut -c1-300 $out/cmp_ab.log
export TMPDIR=/tmp
for lib in head cmph; do
GCK_LIB_PATH=$L/libgocask_hip_$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_$lib -o run -- python3 tools/bench_compact.py > $out/kt_$lib.log 2>&1 || exit 1
python3 - $out/kt_$lib <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].replace("void ", "")
    if "cmp" in n:
        print(f"  {n[:40]:40s} calls {int(r['Calls']):5d} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
done
