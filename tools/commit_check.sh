#!/bin/bash
# One GPU call: the replica commit loop's host phases, kernel phases and a rocprof timeline.
# Usage (via gpurun): bash tools/commit_check.sh <tag>
set -o pipefail
tag=${1:-commit}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for ae in "" "--no-account-events"; do
    timeout -k 10 120 python -u tools/commit_timeline.py --mode 2 $ae >> $out/phases.jsonl || exit 1
    timeout -k 10 120 python -u tools/commit_timeline.py --mode 1 $ae >> $out/phases.jsonl || exit 1
    timeout -k 10 120 python -u tools/commit_timeline.py --mode 0 $ae >> $out/phases.jsonl || exit 1
done
cat $out/phases.jsonl
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/commit_timeline.py \
    --mode 0 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
k=$(find $out/prof -name "*kernel_trace.csv" | head -1)
m=$(find $out/prof -name "*memory_copy_trace.csv" | head -1)
python3 tools/commit_timeline.py --timeline $k $m > $out/timeline.txt
tail -60 $out/timeline.txt
