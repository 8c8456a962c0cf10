#!/bin/bash
# Instruction-fetch PMC passes over configs 3/4 (the flow engine and the account walk are long
# kernels): one pass of SQ wave counters, one of the instruction cache's hits and misses.
# Usage (repo root, via gpurun): bash tools/pmc_icache.sh <tag> <configs>
set -o pipefail
tag=${1:-icache}; cfg=${2:-4}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_SALU" \
            "SQC_ICACHE_HITS SQC_ICACHE_MISSES"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $out/p$i -o run -- \
        python3 $R/tools/bench_configs.py --configs $cfg --no-profile > $out/p$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -5 $out/p$i.log; exit 1; }
done
cd $R && python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
        if k in ("flow_replay", "lanes_walk", "plan_keys", "tr_commit", "group_sort"):
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in tot.items():
    print(k, {n: round(v) for n, v in sorted(c.items())})
PY
