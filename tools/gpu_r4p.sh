set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4p
mkdir -p $out
for v in noboth full; do
  lib=gocask_amd/var/libgocask_hip_$v.so; [ $v = full ] && lib=gocask_amd/libgocask_hip.so
  GCK_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o run -- python3 tools/scrub.py > $out/$v.log 2>&1 || exit $?
  python3 - $out/$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0]
    if any(k in n for k in ("k_verify", "k_scrub", "fill")):
        print(sys.argv[1], n, r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
