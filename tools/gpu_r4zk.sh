set -o pipefail
out=gpurun_out/r4zk
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python tools/copy_ceiling.py > $out/copy.log 2>&1 || { cat $out/copy.log; exit 1; }
tail -1 $out/copy.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex "k_encode_batch" --output-format csv -d $out/pmc_enc_$c -o run -- python3 tools/bench_encode.py --iters 1 > $out/pmc_enc_$c.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex "copy|elementwise" --output-format csv -d $out/pmc_copy_$c -o run -- python3 tools/copy_ceiling.py > $out/pmc_copy_$c.log 2>&1 || exit 1
done
python3 - $out <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in sorted(glob.glob(out + "/pmc_*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in acc.items():
        print(f.split("/")[2], k, c, "dispatch-avg", round(sum(v) / max(1, len(set(v))) if False else sum(v), 1), "n", len(v))
PY
