#!/usr/bin/env python3
"""The flow plan's kernels and the gaps between them, per replayed call, from a rocprofv3
--kernel-trace CSV (e.g. of tools/bench_configs.py --no-profile).

A plan runs from `flow_heads` to the last kernel before the replay proper (`lanes_walk` /
`lanes_replay` / `flow_replay`). Per plan: its wall span on the GPU, the kernels' busy time, the
idle gaps between consecutive kernels (host launch latency the GPU waited on), and the launch
count; then the totals and the mean per plan, and the same for the replay kernels.

Usage: python tools/flow_gaps.py <kernel_trace.csv> [out.json]
"""
import csv
import json
import sys
from collections import defaultdict

REPLAY = ("lanes_walk", "lanes_replay", "flow_replay")


def short(name):
    n = name.split("(")[0].replace("void ", "")
    n = n.split("<")[0]
    return n.split("::")[-1]


def main(path, out=None):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    plans, cur = [], None
    replay = defaultdict(float)
    for s, e, k in rows:
        if k == "flow_heads":
            cur = {"start": s, "end": e, "busy": 0, "launches": 0, "kernels": defaultdict(float),
                   "last_end": s}
            plans.append(cur)
        if cur is None:
            continue
        if k in REPLAY:
            replay[k] += (e - s) / 1e3
            cur = None
            continue
        cur["busy"] += e - s
        cur["launches"] += 1
        cur["kernels"][k] += (e - s) / 1e3
        cur["end"] = max(cur["end"], e)
    n = len(plans)
    if not n:
        print("no flow plans in the trace")
        return
    span = sum(p["end"] - p["start"] for p in plans) / 1e3
    busy = sum(p["busy"] for p in plans) / 1e3
    kern = defaultdict(float)
    for p in plans:
        for k, v in p["kernels"].items():
            kern[k] += v
    res = {"plans": n, "span_us_total": round(span, 1), "busy_us_total": round(busy, 1),
           "gap_us_total": round(span - busy, 1),
           "span_us_per_plan": round(span / n, 1), "busy_us_per_plan": round(busy / n, 1),
           "gap_us_per_plan": round((span - busy) / n, 1),
           "launches_per_plan": round(sum(p["launches"] for p in plans) / n, 1),
           "kernels_us_per_plan": {k: round(v / n, 2) for k, v in
                                   sorted(kern.items(), key=lambda kv: -kv[1])},
           "replay_us_total": {k: round(v, 1) for k, v in replay.items()}}
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
