#!/bin/bash
# GPU parity tests, then config 3 with the walk's debug statistics, then a same-box A/B of the
# walk's deferred verdicts (TBG_WALK_NO_DEFER) on config 3.
set -o pipefail
tag=${1:-walkcheck}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -40 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
TBG_FLOW_DEBUG=1 timeout -k 10 240 python -u tools/bench_configs.py --configs 3 > $out/c3dbg.json 2> $out/c3dbg.err || { tail -5 $out/c3dbg.err; exit 1; }
grep "walk:" $out/c3dbg.err | tail -4
for i in 1 2; do
  for v in defer nodefer; do
    if [ $v = nodefer ]; then export TBG_WALK_NO_DEFER=1; else unset TBG_WALK_NO_DEFER; fi
    timeout -k 10 240 python -u tools/bench_configs.py --configs 3 > $out/$v.$i.json 2> $out/$v.$i.err || { tail -5 $out/$v.$i.err; exit 1; }
    python3 -c "import json,sys
d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['device_transfers_per_s'], d['kernels_ms'].get('tr_lanes'))" $out/$v.$i.json $v.$i
  done
done
