#!/usr/bin/env python3
"""Where the GPU idles inside create_transfers calls, from a rocprofv3 --kernel-trace CSV (e.g. of
tools/bench_configs.py --no-profile).

A call runs from one `tr_chunk_info` (a large call's first kernel) to the last kernel before the
next one. Per call: its span on the GPU, the kernels' busy time, and the idle gaps between
consecutive kernels, each gap charged to the kernel that ended it (the launch the GPU waited
for). Prints the totals per call and the gaps by kernel, largest first.

Usage: python tools/call_gaps.py <kernel_trace.csv> [out.json]
"""
import csv
import json
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0].replace("void ", "")
    n = n.split("<")[0]
    return n.split("::")[-1]


def main(path, out=None):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    calls, cur = [], None
    for s, e, k in rows:
        if k == "tr_chunk_info":
            cur = {"start": s, "end": e, "busy": 0.0, "gaps": defaultdict(float),
                   "busy_by": defaultdict(float), "last_end": s}
            calls.append(cur)
        if cur is None:
            continue
        gap = max(0, s - cur["last_end"])
        if gap:
            cur["gaps"][k] += gap / 1e3
        cur["busy"] += (min(e, max(e, cur["last_end"])) - max(s, cur["last_end"])) / 1e3 \
            if e > cur["last_end"] else 0.0
        cur["busy_by"][k] += (e - s) / 1e3
        cur["last_end"] = max(cur["last_end"], e)
        cur["end"] = cur["last_end"]
    n = len(calls)
    if not n:
        print("no calls in the trace")
        return
    gaps, busy_by = defaultdict(float), defaultdict(float)
    for c in calls:
        for k, v in c["gaps"].items():
            gaps[k] += v
        for k, v in c["busy_by"].items():
            busy_by[k] += v
    span = sum(c["end"] - c["start"] for c in calls) / 1e3
    busy = sum(c["busy"] for c in calls)
    res = {"calls": n, "span_us_per_call": round(span / n, 1),
           "busy_us_per_call": round(busy / n, 1),
           "idle_us_per_call": round((span - busy) / n, 1),
           "idle_before_us_per_call": {k: round(v / n, 2) for k, v in
                                       sorted(gaps.items(), key=lambda kv: -kv[1]) if v / n >= 0.1},
           "kernel_us_per_call": {k: round(v / n, 2) for k, v in
                                  sorted(busy_by.items(), key=lambda kv: -kv[1]) if v / n >= 0.1}}
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
