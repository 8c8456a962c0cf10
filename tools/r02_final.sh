#!/bin/bash
# Round-end evidence: GPU tests, the default bench line with its kernel-trace profile, config 5,
# configs 3/4 (oracle-checked) and the drop-in commit split. Usage: bash tools/r02_final.sh <tag>
set -o pipefail
tag=${1:-final}; out=gpurun_out/$tag
bash tools/gpu_check.sh $tag > gpurun_out/$tag.check.log 2>&1 || { tail -30 gpurun_out/$tag.check.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload config5 --no-cpu-baseline > $out/bench_config5.json 2> $out/bench_config5.err || { tail -5 $out/bench_config5.err; exit 1; }
timeout -k 10 300 python -u tools/bench_configs.py --configs 3,4 > $out/configs34.json 2> $out/configs34.err || { tail -5 $out/configs34.err; exit 1; }
timeout -k 10 300 python -u tools/commit_profile.py --commits 300 > $out/commit_profile.json 2> $out/commit_profile.err || { tail -5 $out/commit_profile.err; exit 1; }
tail -2 $out/gpu_tests.log
python3 - $out <<'PY'
import json, sys
o = sys.argv[1]
b = json.load(open(f"{o}/bench.json"))
print("config2", b["value"], b["roofline"]["frac"], b["roofline"]["path"]["frac"], b["per_commit"]["device"]["us_per_commit_mean"], b["per_commit"]["state_machine"]["us_per_commit_mean"])
c5 = json.load(open(f"{o}/bench_config5.json"))
print("config5", c5["value"], c5["roofline"]["frac"])
for l in open(f"{o}/configs34.json"):
    d = json.loads(l); print(d["config"], d["gpu_transfers_per_s"], d["device_transfers_per_s"])
PY
