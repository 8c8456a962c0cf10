# Same-box A/B of library variants on configs 3/4: the profiled device time (tools/bench_configs.py,
# HIP-event marks) of each variant, twice, interleaved. bash tools/ab_c34.sh <tag> <variant>...
# ("default" = libtbg.so, else tigerbeetle_amd/lib/variants/libtbg_<variant>.so)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
for rep in 1 2; do
  for v in "$@"; do
    lib=""
    [ "$v" = default ] || lib=$PWD/tigerbeetle_amd/lib/variants/libtbg_$v.so
    TBG_LIB=$lib timeout -k 10 300 python3 tools/bench_configs.py $AB_ARGS > $out/c34_${v}_$rep.json 2> $out/c34_${v}_$rep.err || { tail -5 $out/c34_${v}_$rep.err; exit 1; }
    python3 - $out/c34_${v}_$rep.json $v <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    k = d["kernels_ms"]
    print(sys.argv[2], d["config"], "device %.3f ms %.3ge/s" % (d["device_ms"], d["device_transfers_per_s"]),
          "plan %.3f" % k.get("flow_plan", 0), "ae %.3f" % k.get("account_events", 0),
          "host_sync %.3f" % k.get("host_sync", 0), "wall %.3ge/s" % d["gpu_transfers_per_s"])
PY
  done
done
