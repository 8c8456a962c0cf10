#!/bin/bash
# One GPU call: the GPU parity tests, then config 4 (the flow replay's workload) under several
# engine shapes (flow.hpp: lanes per wave x waves x workgroups, XCD packing).
# Usage (from the repo root, via gpurun): bash tools/flow_sweep.sh <tag> [transfers]
set -o pipefail
tag=${1:-flow}; n=${2:-300000}
out=gpurun_out/$tag
mkdir -p $out
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
# SHAPES: "lpw waves blocks xcd_stride" entries separated by commas
IFS=, read -ra shapes <<< "${SHAPES:-64 8 1 1,8 4 16 8,1 8 64 8,1 4 256 1}"
for shape in "${shapes[@]}"; do
    set -- $shape
    echo "shape lpw=$1 waves=$2 blocks=$3 xcd=$4"
    TBG_FLOW_LPW=$1 TBG_FLOW_WAVES=$2 TBG_FLOW_BLOCKS=$3 TBG_FLOW_XCD=$4 \
        timeout -k 10 240 python -u tools/bench_configs.py --configs 4 --transfers $n \
        > $out/c4_$1_$2_$3_$4.json 2> $out/c4_$1_$2_$3_$4.err || { tail -5 $out/c4_$1_$2_$3_$4.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['gpu_transfers_per_s'], d['oracle_transfers_per_s'], d['kernels_ms'].get('tr_flow'))" $out/c4_$1_$2_$3_$4.json
done
