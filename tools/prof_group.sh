#!/bin/bash
# Kernel statistics of bench.py's group rehearsal (a group of S shards on one GPU) under
# rocprofv3 --kernel-trace --stats. Usage (repo root, via gpurun): bash tools/prof_group.sh <tag> [S]
set -o pipefail
tag=${1:-group}
S=${2:-2}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --group $S --steps 5 --warmup 1 > $out/run.json 2> $out/run.err || exit 1
cd $GRAFT_REPO_ROOT

python3 - "$out" <<'PY'
import csv, glob, sys
out = sys.argv[1]
f = glob.glob(f"{out}/prof/**/run_kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
with open(f"{out}/kernel_stats.txt", "w") as o:
    for r in rows[:45]:
        name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        line = f'{name[:60]:60s} {int(r["Calls"]):6d} {float(r["TotalDurationNs"])/1e3:10.1f} us {float(r["AverageNs"])/1e3:9.2f} us avg'
        print(line)
        o.write(line + "\n")
PY
