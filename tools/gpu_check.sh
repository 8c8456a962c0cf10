#!/bin/bash
# One GPU call: parity tests, a bench line and a kernel-trace profile of the bench's timed steps.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh <tag> [bench args...]
#   TBG_SKIP_TESTS=1 skips the pytest step.
set -o pipefail
tag=${1:-run}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ -z "$TBG_SKIP_TESTS" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        --durations=12 > $out/gpu_tests.log 2>&1 || { tail -40 $out/gpu_tests.log; exit 1; }
    tail -16 $out/gpu_tests.log
fi
timeout -k 10 300 python -u bench.py "$@" > $out/bench.json 2> $out/bench.err || { cat $out/bench.err; exit 1; }
cat $out/bench.json
# The profile covers the bench's own steps only (no per-commit calls, no CPU baseline, no hazard
# call -- the group's shards run smaller tr_ingest launches): its
# tr_ingest launches are all full 10M-event steps, comparable with roofline.avg_launch_ms.
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --commit-reps 0 --no-account-events-line --no-hazard-call "$@" > $GRAFT_REPO_ROOT/$out/prof_bench.json 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
trace=$(find $out/prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py $trace $out/trace_summary.json tr_ingest
