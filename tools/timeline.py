#!/usr/bin/env python3
"""One replay step as a timeline, from a rocprofv3 --kernel-trace CSV:
every dispatch between a k_run_init and the next k_publish, its duration and
the idle gap before it (device clock), median over the steps found.

  python tools/timeline.py gpurun_out/kt_<tag>      -> one JSON line
"""
import csv
import glob
import json
import statistics
import sys


def main():
    root = sys.argv[1]
    f = [p for p in glob.glob(root + "/**/*kernel_trace.csv", recursive=True)][0]
    rows = list(csv.DictReader(open(f)))
    ks = []
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ks.append((s, e, name.split("(")[0].replace("void ", "").replace("gck::", "")))
    ks.sort()
    steps, cur = [], None
    for s, e, n in ks:
        if n.startswith("k_run_init"):
            cur = [(s, e, n)]
        elif cur is not None:
            cur.append((s, e, n))
            if n.startswith("k_publish"):
                steps.append(cur)
                cur = None
    per = {}
    spans = []
    for st in steps:
        spans.append((st[-1][1] - st[0][0]) / 1e3)
        prev_end = st[0][0]
        for i, (s, e, n) in enumerate(st):
            key = f"{i:02d} {n}"
            d = per.setdefault(key, dict(dur=[], gap=[]))
            d["dur"].append((e - s) / 1e3)
            d["gap"].append((s - prev_end) / 1e3)
            prev_end = e
    out = dict(steps=len(steps), span_us_median=round(statistics.median(spans), 1) if spans else None,
               kernels={k: dict(us=round(statistics.median(v["dur"]), 1), gap_us=round(statistics.median(v["gap"]), 1))
                        for k, v in sorted(per.items())})
    tot_gap = sum(v["gap_us"] for v in out["kernels"].values())
    out["gaps_us_total"] = round(tot_gap, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
