# Kernel trace of tools/kd_time.py (C3 keydir builds): per-kernel averages.
#   bash tools/kd_ktrace.sh <tag>   -> gpurun_out/kt_<tag>/
set -o pipefail
tag=${1:-kd}
export TMPDIR=/tmp
out=gpurun_out/kt_$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
  python3 tools/kd_time.py > $out/kd_time.log 2>&1 || exit $?
python3 - "$out" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].replace("void ", "")
    print(f"{n[:48]:48s} calls {int(r['Calls']):5d} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
