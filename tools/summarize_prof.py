"""Condense a tools/pmc.sh run (gpurun_out/prof_<tag>/) into profiles/<tag>/.

  python tools/summarize_prof.py <tag> [config]

Writes
  profiles/<tag>/kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<tag>/pmc_summary.json   per-kernel mean of every PMC counter, per dispatch
  profiles/<tag>/bench.json         the bench line printed under the trace pass
  profiles/traffic_<config>.json    k_crc_rows HBM bytes per launch, read by bench.py

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and, on gfx950,
reports half of the bytes of a 16 B/lane streaming read, so bytes = FETCH_SIZE
x 1024 x 2.  The k_stream_read dispatches of the same run (a plain read of the
whole arena) calibrate that factor: their corrected bytes must equal the arena.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("gck::", "")


def main():
    tag = sys.argv[1]
    cfg = sys.argv[2] if len(sys.argv) > 2 else "c3"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    bench = None
    for line in open(os.path.join(src, "trace.log")):
        if line.startswith("{"):
            bench = json.loads(line)
    if bench:
        json.dump(bench, open(os.path.join(dst, "bench.json"), "w"), indent=1)
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    i = 1
    while os.path.exists(os.path.join(src, f"pmc{i}", "run_counter_collection.csv")):
        for r in csv.DictReader(open(os.path.join(src, f"pmc{i}", "run_counter_collection.csv"))):
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        i += 1
    summary = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in pmc.items()}
    json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1, sort_keys=True)
    stats = {}
    for r in csv.DictReader(open(os.path.join(dst, "kernel_stats.csv"))):
        stats[short(r["Name"])] = float(r["AverageNs"])
    crc_key = next((k for k in summary if (k == "k_crc_rows" or k.startswith("k_crc_rows<"))), None)
    crc = summary.get(crc_key, {})
    sr = next((v for k, v in summary.items() if k.startswith("k_stream_read")), {})
    out = {
        "config": cfg,
        "source": f"profiles/{tag}/pmc_summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
        "correction": "bytes = FETCH_SIZE[KiB] * 1024 * 2 (gfx950 wide streaming reads, MI355X_MICROARCH.md HBM)",
        "crc_rows_hbm_bytes_per_launch": crc.get("FETCH_SIZE", 0) * 2048 or None,
        "crc_rows_write_bytes_per_launch": crc.get("WRITE_SIZE", 0) * 1024 or None,
        "stream_read_hbm_bytes_per_launch": sr.get("FETCH_SIZE", 0) * 2048 or None,
        "crc_rows_avg_ns_rocprof": next((v for k, v in stats.items() if (k == "k_crc_rows" or k.startswith("k_crc_rows<"))), None),
        "algorithmic_bytes_per_launch": (bench["config"]["bytes_per_gpu"] / bench["roofline"].get("launches_per_step", 1))
        if bench else None,
    }
    json.dump(out, open(os.path.join(ROOT, "profiles", f"traffic_{cfg}.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
