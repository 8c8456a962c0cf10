#!/bin/bash
# GPU tests + configs 3/4 with the flow engine's per-call statistics (TBG_FLOW_DEBUG).
set -o pipefail
tag=${1:-c34dbg}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/gpu_tests.log 2>&1 || { tail -60 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
timeout -k 10 300 python -u tools/bench_configs.py --configs 3,4 > $out/configs34.json 2> $out/configs34.err || { tail -30 $out/configs34.err; exit 1; }
cat $out/configs34.json
TBG_FLOW_DEBUG=1 timeout -k 10 300 python -u tools/bench_configs.py --configs 3,4 > $out/configs34_dbg.json 2> $out/flow_debug.txt || { tail -30 $out/flow_debug.txt; exit 1; }
grep -c flow: $out/flow_debug.txt
