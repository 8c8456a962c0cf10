#!/bin/bash
# One GPU call: the default bench line, configs 3/4 against the oracle (with per-kernel device
# times), config 4 without profiling (production paths: the AccountEvents behind the next call,
# host-timed pulses), and a summary. Usage (repo root, via gpurun): bash tools/measure.sh <tag>
set -o pipefail
tag=${1:-measure}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
timeout -k 10 500 python -u tools/bench_configs.py --configs 3,4 > $out/configs34.json 2> $out/configs34.err || { tail -20 $out/configs34.err; exit 1; }
timeout -k 10 300 python -u tools/bench_configs.py --configs 4 --no-profile > $out/config4_noprof.json 2> $out/config4_noprof.err || { tail -20 $out/config4_noprof.err; exit 1; }
python3 - "$out" <<'EOF'
import json, sys
out = sys.argv[1]
for f in ("configs34", "config4_noprof"):
    for l in open(f"{out}/{f}.json"):
        if l.startswith("{"):
            d = json.loads(l)
            print(f, d["config"], d["validated"], d.get("device_transfers_per_s"),
                  d["gpu_transfers_per_s"], d["pulse"])
            if d.get("kernels_ms"):
                print("   ", d["kernels_ms"])
d = json.loads(open(f"{out}/bench.json").read().strip().splitlines()[-1])
pc = d["per_commit"]
print("config2", d["value"], "with_ae", d["with_account_events"]["value"],
      "sm_us mean/p50", pc["state_machine"]["us_per_commit_mean"],
      pc["state_machine"]["us_per_commit_p50"], "device_us", pc["device"]["us_per_commit_mean"])
print("   ", d["with_account_events"]["kernels_ms_per_step"])
EOF
