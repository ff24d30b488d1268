# Kernel traces of the bench for several library builds on one box:
#   bash tools/kt_ab.sh <tag> lib1.so lib2.so ...   -> gpurun_out/ktab_<tag>/
set -o pipefail
tag=${1:-x}; shift
export TMPDIR=/tmp
out=gpurun_out/ktab_$tag
mkdir -p $out
i=0
for lib in "$@"; do
  i=$((i+1))
  echo "== $lib"
  GCK_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/t$i -o run -- \
    python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --verbose > $out/bench$i.json 2> $out/bench$i.err || exit $?
  python3 - "$out/t$i" "$out/bench$i.json" <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].replace("void ", "")
    if float(r['AverageNs']) > 20e3 and 'encode' not in n and 'fill' not in n:
        print(f"  {n[:40]:40s} calls {int(r['Calls']):5d} avg_us {float(r['AverageNs'])/1e3:9.1f}")
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("  step", d['ms_per_step'], "fixups", d.get('fixups'), {k: round(v, 3) for k, v in d['phase_ms'].items()})
PY
done
