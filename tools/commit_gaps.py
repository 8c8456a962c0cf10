#!/usr/bin/env python3
"""Per small create_transfers call (one replica commit), its kernels and the GPU idle time between
them, from a rocprofv3 --kernel-trace CSV of bench.py's `per_commit` (or tools/commit_timeline.py).

A commit starts at a `tr_ingest` launch of at most `--max-grid` work-items and runs to the next
one; the report gives the mean span (first kernel start to last kernel end), busy time, idle gaps,
launches, each kernel's mean duration, and the mean distance between consecutive commits' starts.

Usage: python tools/commit_gaps.py <kernel_trace.csv> [--max-grid 65536] [--skip 10] [--out f.json]
"""
import argparse
import csv
import json
from collections import defaultdict


def short(name):
    n = name.split("(")[0].replace("void ", "").split("<")[0]
    return n.split("::")[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--max-grid", type=int, default=65536)
    ap.add_argument("--skip", type=int, default=10, help="commits skipped at the start (warmup)")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                     int(r["Grid_Size_X"])))
    rows.sort()
    commits, cur = [], None
    for s, e, k, g in rows:
        if k == "tr_ingest":
            cur = None
            if g <= a.max_grid:
                cur = {"start": s, "end": e, "busy": 0, "kernels": defaultdict(float), "n": 0}
                commits.append(cur)
        if cur is None:
            continue
        cur["end"] = max(cur["end"], e)
        cur["busy"] += e - s
        cur["n"] += 1
        cur["kernels"][k] += (e - s) / 1e3
    commits = commits[a.skip:]
    if not commits:
        print("no commits found")
        return
    n = len(commits)
    span = sum(c["end"] - c["start"] for c in commits) / n / 1e3
    busy = sum(c["busy"] for c in commits) / n / 1e3
    starts = [c["start"] for c in commits]
    period = (starts[-1] - starts[0]) / (n - 1) / 1e3 if n > 1 else None
    kern = defaultdict(float)
    for c in commits:
        for k, v in c["kernels"].items():
            kern[k] += v / n
    res = {"commits": n, "span_us": round(span, 2), "busy_us": round(busy, 2),
           "gap_us": round(span - busy, 2), "launches": round(sum(c["n"] for c in commits) / n, 2),
           "start_to_start_us": round(period, 2) if period else None,
           "kernels_us": {k: round(v, 2) for k, v in sorted(kern.items(), key=lambda kv: -kv[1])}}
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
