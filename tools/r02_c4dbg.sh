#!/bin/bash
# Config 4 with the flow engine's per-call statistics and critical path (TBG_FLOW_DEBUG).
set -o pipefail
tag=${1:-c4dbg}; out=gpurun_out/$tag; mkdir -p $out
TBG_FLOW_DEBUG=1 timeout -k 10 300 python -u tools/bench_configs.py --configs ${CONFIGS:-4} > $out/configs_dbg.json 2> $out/flow_debug.txt || { tail -30 $out/flow_debug.txt; exit 1; }
grep -E "flow: (m=|critical)" $out/flow_debug.txt | tail -16
