#!/bin/bash
# Config 4 flow engine at several engine shapes (LPW WAVES BLOCKS), with per-call debug statistics.
set -o pipefail
tag=${1:-lanesweep}; out=gpurun_out/$tag; mkdir -p $out
for shape in "1 1 1" "1 1 64" "1 1 256" "8 4 256"; do
  set -- $shape
  n="$1_$2_$3"
  TBG_FLOW_DEBUG=1 TBG_FLOW_LPW=$1 TBG_FLOW_WAVES=$2 TBG_FLOW_BLOCKS=$3 timeout -k 10 240 python -u tools/bench_configs.py --configs 4 > $out/$n.json 2> $out/$n.err || { tail -5 $out/$n.err; exit 1; }
  echo "== $n"; grep -E "flow: (m=|critical)" $out/$n.err | head -4
  python3 -c "import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); k=d['kernels_ms']; print(d['config'], d['gpu_transfers_per_s'], k.get('tr_flow'), k.get('flow_plan'))" $out/$n.json
done
