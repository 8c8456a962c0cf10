set -o pipefail
out=gpurun_out/r02_i; mkdir -p $out
TBG_FLOW_DEBUG=1 timeout -k 10 300 python -u tools/bench_configs.py --configs 3 > $out/configs.json 2> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
grep walk: $out/configs.err | head -20
