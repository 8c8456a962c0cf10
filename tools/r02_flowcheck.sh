#!/bin/bash
# GPU parity tests, then config 4 (flow engine) with debug statistics at the default shape and
# with one lane (per-event latency without contention), then configs 3/4 timing.
set -o pipefail
tag=${1:-flowcheck}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -40 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
for shape in "1 1 1" "8 4 256"; do
  set -- $shape
  n="$1_$2_$3"
  TBG_FLOW_DEBUG=1 TBG_FLOW_LPW=$1 TBG_FLOW_WAVES=$2 TBG_FLOW_BLOCKS=$3 timeout -k 10 240 python -u tools/bench_configs.py --configs 4 > $out/$n.json 2> $out/$n.err || { tail -5 $out/$n.err; exit 1; }
  echo "== $n"; grep -E "flow: (m=|critical)" $out/$n.err | head -4
done
timeout -k 10 240 python -u tools/bench_configs.py --configs 3,4 > $out/configs.json 2> $out/configs.err || { tail -5 $out/configs.err; exit 1; }
python3 -c "import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); k=d['kernels_ms']; print(d['config'], d['gpu_transfers_per_s'], d.get('device_transfers_per_s'), k.get('tr_flow'), k.get('tr_lanes'), k.get('flow_plan'))" $out/configs.json
