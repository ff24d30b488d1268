set -o pipefail
out=gpurun_out/r4zz
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_get.py tests/test_gpu_encode_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { tail -5 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 tools/scrub.py > $out/kt.log 2>&1 || { tail $out/kt.log; exit 1; }
grep scrub_ms $out/kt.log
python3 - $out <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].replace("void ", "")
    if any(k in n for k in ("verify", "scrub")):
        print(f"  {n[:40]:40s} calls {int(r['Calls']):5d} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
for c in FETCH_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex "k_verify" --output-format csv -d $out/pmc_$c -o run -- python3 tools/scrub.py > $out/pmc_$c.log 2>&1 || exit 1
done
python3 - $out <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/pmc_*/**/*counter_collection.csv", recursive=True):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))]
    print(f.split("/")[2], "per dispatch KiB", sum(v) / 3)
PY
