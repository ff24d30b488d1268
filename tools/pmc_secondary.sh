# One PMC pass each over the encoder and the scrub (tools/bench_encode.py,
# tools/scrub.py): instruction mix and stall counters of their kernels.
#   bash tools/pmc_secondary.sh <tag>   -> gpurun_out/pmcs_<tag>/
set -o pipefail
tag=${1:-x}
export TMPDIR=/tmp
out=gpurun_out/pmcs_$tag
mkdir -p $out
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
timeout -k 10 120 rocprofv3 --pmc $C --kernel-include-regex "k_encode_batch" --output-format csv -d $out/enc -o run -- \
  python3 tools/bench_encode.py > $out/enc.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc $C --kernel-include-regex "k_verify" --output-format csv -d $out/scrub -o run -- \
  python3 tools/scrub.py > $out/scrub.log 2>&1 || exit $?
# (FETCH_SIZE and WRITE_SIZE need 3 + 2 TCC counters: one run each)
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_encode_batch" --output-format csv -d $out/fetch -o run -- \
  python3 tools/bench_encode.py > $out/fetch.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_encode_batch" --output-format csv -d $out/write -o run -- \
  python3 tools/bench_encode.py > $out/write.log 2>&1 || exit $?
python3 - "$out" <<'PY'
import csv, glob, sys, collections
for sub in ("enc", "scrub", "fetch", "write"):
    f = glob.glob(f"{sys.argv[1]}/{sub}/**/*counter_collection.csv", recursive=True)
    if not f: continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        print(sub, k[:40], {c: round(x / 1e6, 2) for c, x in sorted(v.items())})
PY
