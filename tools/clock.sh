# Effective shader clock per kernel: GRBM_GUI_ACTIVE (GPU-busy clock cycles) / kernel duration.
#   bash tools/clock.sh <tag>  -> gpurun_out/clk_<tag>/
set -o pipefail
tag=${1:-x}
export TMPDIR=/tmp
out=gpurun_out/clk_$tag
mkdir -p $out
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "k_crc_rows|k_stream_read|k_finalize|k_walk" \
  --output-format csv -d $out -o run -- python3 tools/ablate.py c3 0,8 > $out/log.txt 2>&1 || exit $?
python3 - "$out" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) if "End_Timestamp" in r else None
    agg[n][r["Counter_Name"]].append((float(r["Counter_Value"]), d))
for n, cs in agg.items():
    for c, v in cs.items():
        vals = [x for x, _ in v]
        ds = [d for _, d in v if d]
        s = f"{n[:32]:32s} {c:16s} n={len(vals)} avg={sum(vals)/len(vals):.4g}"
        if ds and c == "GRBM_GUI_ACTIVE":
            s += f" dur_ns={sum(ds)/len(ds):.0f} -> {sum(vals)/sum(ds):.3f} GHz"
        print(s)
PY
