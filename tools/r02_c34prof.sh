#!/bin/bash
# Configs 3/4 under rocprofv3 --kernel-trace --stats (oracle-checked), kernel summary to stdout.
set -o pipefail
tag=${1:-c34prof}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs ${CONFIGS:-3,4} > $GRAFT_REPO_ROOT/$out/configs.json 2> $GRAFT_REPO_ROOT/$out/configs.err || exit 1
cd $GRAFT_REPO_ROOT && find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
cat $out/configs.json
python3 - $out/kernel_stats.csv <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:28]:
    n = re.sub(r'rocprim::ROCPRIM_400200_NS::', '', r['Name'])[:90]
    print(r['Calls'].rjust(5), str(int(r['TotalDurationNs']) // 1000).rjust(7), 'us', str(round(float(r['AverageNs']) / 1000, 1)).rjust(7), n)
PY
