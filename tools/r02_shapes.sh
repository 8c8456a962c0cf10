#!/bin/bash
# Config 4 create_transfers device time at several flow-engine shapes (LPW WAVES BLOCKS).
set -o pipefail
tag=${1:-shapes}; out=gpurun_out/$tag; mkdir -p $out
for shape in ${SHAPES_LIST:-"8 4 256" "4 4 512" "2 4 1024" "4 4 256" "2 4 512" "1 4 1024"}; do
  set -- $shape
  n="$1_$2_$3"
  TBG_FLOW_LPW=$1 TBG_FLOW_WAVES=$2 TBG_FLOW_BLOCKS=$3 timeout -k 10 240 python -u tools/bench_configs.py --configs 4 > $out/$n.json 2> $out/$n.err || { tail -5 $out/$n.err; exit 1; }
  python3 -c "import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); k=d['kernels_ms']; print(sys.argv[2], d['device_transfers_per_s'], k.get('tr_flow'))" $out/$n.json $n
done
