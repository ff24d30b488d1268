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
# memory-side passes: L2 hits, TA / TD busy and the shader clock, L2 read latency
i=0
for C2 in "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
          "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C2 --kernel-include-regex "k_encode_batch" --output-format csv -d $out/enc_m$i -o run -- \
    python3 tools/bench_encode.py > $out/enc_m$i.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc $C2 --kernel-include-regex "k_verify" --output-format csv -d $out/scrub_m$i -o run -- \
    python3 tools/scrub.py > $out/scrub_m$i.log 2>&1 || exit $?
done
# (FETCH_SIZE and WRITE_SIZE need 3 + 2 TCC counters: one run each)
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_encode_batch" --output-format csv -d $out/fetch -o run -- \
  python3 tools/bench_encode.py > $out/fetch.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_encode_batch" --output-format csv -d $out/write -o run -- \
  python3 tools/bench_encode.py > $out/write.log 2>&1 || exit $?
python3 - "$out" <<'PY'
import csv, glob, sys, collections, json
summary = {}
for sub in ("enc", "scrub", "enc_m1", "scrub_m1", "enc_m2", "scrub_m2", "fetch", "write"):
    f = glob.glob(f"{sys.argv[1]}/{sub}/**/*counter_collection.csv", recursive=True)
    if not f: continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, v in acc.items():
        n = len(disp[k])
        row = summary.setdefault(k, {"dispatches": n})
        row.update({c: x / n for c, x in v.items()})
        row.setdefault("us_per_dispatch", sum(disp[k].values()) / n / 1e3)
for k, row in summary.items():
    wc = row.get("SQ_WAVE_CYCLES")
    d = {}
    if wc:
        d.update(wait=row["SQ_WAIT_ANY"] / wc, issue_stall=row["SQ_WAIT_INST_ANY"] / wc,
                 busy=1 - (row["SQ_WAIT_ANY"] + row["SQ_WAIT_INST_ANY"]) / wc)
    if "GRBM_GUI_ACTIVE" in row:
        cyc = row["GRBM_GUI_ACTIVE"] / 8  # (summed over the 8 XCDs)
        d.update(ghz=cyc / (row["us_per_dispatch"] * 1e3), ta_busy=row["TA_TA_BUSY_sum"] / (cyc * 256),
                 td_busy=row["TD_TD_BUSY_sum"] / (cyc * 256),
                 l2_hit=row["TCC_HIT_sum"] / max(1.0, row["TCC_HIT_sum"] + row["TCC_MISS_sum"]))
    if row.get("TCP_TCC_READ_REQ_sum"):
        d["l2_read_latency_cycles"] = row["TCP_TCC_READ_REQ_LATENCY_sum"] / row["TCP_TCC_READ_REQ_sum"]
    row["derived"] = {a: round(b, 3) for a, b in d.items()}
    print(k[:40], json.dumps(row["derived"]), "us", round(row["us_per_dispatch"], 1))
json.dump(summary, open(sys.argv[1] + "/summary.json", "w"), indent=1)
PY
