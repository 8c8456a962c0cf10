#!/bin/bash
# Same-box A/B of a flow-replay knob on config 4 (and 3): runs alternate the default and the knob.
# Usage: KNOB=TBG_FLOW_NO_PREFETCH bash tools/r02_ab_flow.sh <tag>
set -o pipefail
tag=${1:-abflow}; out=gpurun_out/$tag; mkdir -p $out
for i in 1 2; do
  for v in default knob; do
    if [ $v = knob ]; then export $KNOB=${KNOBVAL:-1}; else unset $KNOB; fi
    timeout -k 10 240 python -u tools/bench_configs.py --configs ${CONFIGS:-4} > $out/$v.$i.json 2> $out/$v.$i.err || { tail -5 $out/$v.$i.err; exit 1; }
    python3 -c "import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); k=d['kernels_ms']; print(sys.argv[2], d['config'], d['gpu_transfers_per_s'], k.get('tr_flow'), k.get('tr_lanes'), k.get('flow_plan'))" $out/$v.$i.json $v.$i
  done
done
