#!/bin/bash
# Round-end evidence in one GPU call: the GPU tests, the default bench line, a kernel-trace profile
# of the bench's timed steps (tools/gpu_check.sh) and configs 3/4 against the oracle.
# Usage (repo root, via gpurun): bash tools/final_check.sh <tag>
set -o pipefail
tag=${1:-final}
bash tools/gpu_check.sh $tag || exit 1
out=gpurun_out/$tag
timeout -k 10 400 python -u tools/bench_configs.py --configs 3,4 > $out/configs34.json 2>&1 || { tail -20 $out/configs34.json; exit 1; }
timeout -k 10 400 python -u tools/bench_configs.py --configs 3,4 --amounts wide > $out/configs34_wide.json 2>&1 || { tail -20 $out/configs34_wide.json; exit 1; }
python3 -c "
import json
for l in list(open('$out/configs34.json')) + list(open('$out/configs34_wide.json')):
    if l.startswith('{'):
        d=json.loads(l); print(d['config'], d['amounts'], d['validated'], d['device_transfers_per_s'], d['gpu_transfers_per_s'], d['replayed'])
"
