#!/usr/bin/env python3
"""Per-launch kernel durations from a rocprofv3 --kernel-trace CSV (the file kept under profiles/).

Usage: python tools/trace_summary.py <run_kernel_trace.csv> <out.json> [kernel substrings...]

Writes, per kernel (short name), the launch count, mean / min / max microseconds and grid size;
for each kernel named on the command line (default: tr_ingest), every launch's duration in
dispatch order -- so that bench.py's `roofline.avg_launch_ms` (HIP events on the executor's
stream) can be checked against the profiler's own clock from a tracked file.
"""
import csv
import json
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    n = n.replace("void ", "")
    return n.split("::")[-1] if "tbg::" in n and "<" not in n else n


def main(path, out, wanted):
    launches = defaultdict(list)
    for row in csv.DictReader(open(path)):
        k = short(row["Kernel_Name"])
        us = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
        launches[k].append((int(row["Dispatch_Id"]), us, int(row["Grid_Size_X"])))
    summary = {}
    for k, v in sorted(launches.items(), key=lambda kv: -sum(x[1] for x in kv[1])):
        us = [x[1] for x in v]
        summary[k] = {"launches": len(v), "total_us": round(sum(us), 1),
                      "mean_us": round(sum(us) / len(us), 2), "min_us": round(min(us), 2),
                      "max_us": round(max(us), 2),
                      "grid_sizes": sorted(set(x[2] for x in v))[:8]}
    per_launch = {}
    for w in wanted:
        for k, v in launches.items():
            if w in k:
                per_launch[k] = [{"dispatch": d, "us": round(us, 2), "grid": g}
                                 for d, us, g in sorted(v)]
    json.dump({"source": path, "kernels": summary, "per_launch": per_launch}, open(out, "w"),
              indent=1)
    for k, d in list(summary.items())[:12]:
        print(f"{k[:60]:60s} {d['launches']:6d} {d['mean_us']:10.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:] or ["tr_ingest"])
