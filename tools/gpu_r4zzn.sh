set -o pipefail
out=gpurun_out/r4zzn
mkdir -p $out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_cmp_copy|k_encode_batch" --output-format csv -d $out/pmc_cmp_$c -o run -- python3 tools/bench_compact.py > $out/pmc_cmp_$c.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_encode_batch" --output-format csv -d $out/pmc_enc_$c -o run -- python3 tools/bench_encode.py --iters 1 > $out/pmc_enc_$c.log 2>&1 || exit 1
done
python3 - $out <<'PY'
import csv, glob, sys, collections, json
res = {}
for f in sorted(glob.glob(sys.argv[1] + "/pmc_*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in acc.items():
        res[f"{f.split('/')[2]}:{k}:{c}"] = {"dispatch_values_kib": v}
print(json.dumps(res, indent=1))
PY
