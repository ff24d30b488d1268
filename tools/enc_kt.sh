# Kernel times of the encoder benchmark under each library build:
#   bash tools/enc_kt.sh lib1.so lib2.so ...   -> gpurun_out/enckt_<n>/
set -o pipefail
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1)); out=gpurun_out/enckt_$i; mkdir -p $out
  GCK_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
    python3 tools/bench_encode.py > $out/bench.log 2>&1 || exit $?
  echo "LIB=$lib"
  python3 - "$out" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].replace("void ", "")
    if "enc" in n:
        print(f"  {n[:40]:40s} calls {int(r['Calls']):5d} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
done
