"""Summarise tools/pmc.sh passes: per kernel, the average per launch of every counter collected.

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived counters). MI355X_MICROARCH.md (HBM): on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so `hbm_read_bytes` doubles
it; WRITE_SIZE is exact for 16-B-per-lane stores. Both include Infinity-Cache-served requests.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    n = name.split("(")[0]
    for key in ("tr_ingest", "tr_commit", "bal_hash_apply", "bal_bucket_scatter",
                "bal_bucket_accumulate", "bal_bucket_apply", "onesweep_iteration",
                "onesweep_global_offsets", "acc_prepare", "acc_classify", "replay_kernel"):
        if key in name:
            return key
    return n[-60:]


def traffic(summary, source):
    """Per-launch HBM bytes of each kernel (the `roofline.traffic` bench.py reports)."""
    ks = {}
    for k, d in summary.items():
        if "hbm_bytes" in d:
            ks[k] = {"hbm_bytes_per_launch": d["hbm_bytes"], "read_bytes": d["hbm_read_bytes"],
                     "write_bytes": d["hbm_write_bytes"], "launches": d.get("FETCH_SIZE_launches")}
    return {"source": source, "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE, "
                                        "separate passes, average per launch", "kernels": ks}


def main(out, traffic_path=None):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"),
                              recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                acc[k][row["Counter_Name"]].append((row["Dispatch_Id"], float(row["Counter_Value"])))
    summary = {}
    for k, ctrs in acc.items():
        d = {}
        for c, vals in ctrs.items():
            per = defaultdict(float)
            for disp, v in vals:
                per[disp] += v
            d[c] = sum(per.values()) / len(per)
            d[c + "_launches"] = len(per)
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes"] = d["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in d and "hbm_write_bytes" in d:
            d["hbm_bytes"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
        summary[k] = d
    json.dump(summary, sys.stdout, indent=1, sort_keys=True)
    print()
    if traffic_path:
        with open(traffic_path, "w") as fh:
            json.dump(traffic(summary, os.path.basename(os.path.normpath(out))), fh, indent=1,
                      sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
