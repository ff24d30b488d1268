set -o pipefail
out=gpurun_out/r4zzk
mkdir -p $out
export TMPDIR=/tmp
cat > $out/kd.py <<'PY'
import os, sys
sys.path.insert(0, os.getcwd())
import gocask_amd as g, bench
ctx = g.ReplayContext()
ctx.encode(**bench.CONFIGS["c3"])
ctx.run()
for _ in range(3):
    n, ms = ctx.keydir(fetch=False)
    print("keydir_ms", round(ms, 3), "live", n, flush=True)
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 $out/kd.py > $out/kt.log 2>&1 || { tail $out/kt.log; exit 1; }
grep keydir_ms $out/kt.log
python3 - $out <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].replace("void ", "")
    if "kd" in n:
        print(f"  {n[:40]:40s} calls {int(r['Calls']):5d} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
