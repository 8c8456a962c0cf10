#!/bin/bash
# GPU tests, then configs 3/4 (oracle-checked) with kernel stats. Usage: bash tools/r02_plan.sh <tag>
set -o pipefail
tag=${1:-plan}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/gpu_tests.log 2>&1 || { tail -60 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
timeout -k 10 300 python -u tools/bench_configs.py --configs 3,4 > $out/configs34.json 2> $out/configs34.err || { tail -30 $out/configs34.err; exit 1; }
cat $out/configs34.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs 3,4 > $GRAFT_REPO_ROOT/$out/prof_configs.json 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
cut -d, -f1-4 $out/kernel_stats.csv | cut -c1-140 | head -30
