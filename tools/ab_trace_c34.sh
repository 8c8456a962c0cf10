# Same-box A/B of library variants on configs 3/4 under a kernel trace (per-kernel durations, no
# HIP-event marks): bash tools/ab_trace_c34.sh <tag> <variant>... ("default" = libtbg.so, else
# tigerbeetle_amd/lib/variants/libtbg_<variant>.so); then tools/flow_gaps.py on each trace.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  lib=""
  [ "$v" = default ] || lib=$PWD/tigerbeetle_amd/lib/variants/libtbg_$v.so
  TBG_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace_$v -- python3 tools/bench_configs.py --configs 3,4 --no-profile > $out/c34_$v.json 2> $out/c34_$v.err || { tail -5 $out/c34_$v.err; exit 1; }
  python3 tools/flow_gaps.py $out/trace_$v/*/*kernel_trace.csv > $out/flow_gaps_$v.json
  echo "$v $(grep -o '"span_us_per_plan": [0-9.]*' $out/flow_gaps_$v.json) $(grep -o '"plan_keys": [0-9.]*' $out/flow_gaps_$v.json)"
done
