set -o pipefail
out=gpurun_out/r4zp
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_get.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $out/pytest.log | head -20; exit $rc; }
L=gocask_amd/var
bash tools/scrub_ab.sh $L/libgocask_hip_encwide.so $L/libgocask_hip_sord3.so > $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
bash tools/scrub_ab.sh $L/libgocask_hip_encwide.so $L/libgocask_hip_sord3.so >> $out/scrub_ab.log 2>&1 || { cat $out/scrub_ab.log; exit 1; }
cat $out/scrub_ab.log
export TMPDIR=/tmp
GCK_LIB_PATH=gocask_amd/var/libgocask_hip_sord3.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 tools/scrub.py > $out/kt.log 2>&1 || { tail $out/kt.log; exit 1; }
python3 - $out <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].replace("void ", "")
    if any(k in n for k in ("verify", "group", "scrub")):
        print(f"  {n[:40]:40s} calls {int(r['Calls']):5d} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
