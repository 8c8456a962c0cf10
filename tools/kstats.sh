#!/bin/bash
# Kernel statistics (rocprofv3 --kernel-trace --stats) of tools/bench_configs.py on the given
# configs, without the per-kernel profiling syncs. Usage (repo root, via gpurun):
#   bash tools/kstats.sh <tag> <configs>
set -o pipefail
tag=${1:-kstats}
cfg=${2:-3,4}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs $cfg --no-profile > $out/run.json 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 - "$out" <<'PY'
import csv, glob, sys
out = sys.argv[1]
f = glob.glob(f"{out}/prof/**/run_kernel_stats.csv", recursive=True) or glob.glob(f"{out}/prof/run_kernel_stats.csv")
rows = list(csv.DictReader(open(f[0])))
with open(f"{out}/kernel_stats.txt", "w") as o:
    for r in rows[:45]:
        name = r["Name"].split("(")[0].replace("void ", "")
        line = f'{name[:60]:60s} {int(r["Calls"]):6d} {float(r["TotalDurationNs"])/1e3:10.1f} us {float(r["AverageNs"])/1e3:9.2f} us avg'
        print(line)
        o.write(line + "\n")
PY
