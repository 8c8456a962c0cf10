set -o pipefail
out=gpurun_out/r06_gaps; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in 3 4; do
  rm -rf $out/trace_c$c
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace_c$c -- python3 tools/bench_configs.py --configs $c ${GAPS_ARGS---no-profile} > $out/c$c.json 2> $out/c$c.err || { tail -5 $out/c$c.err; exit 1; }
  python3 tools/call_gaps.py $out/trace_c$c/*/*kernel_trace.csv $out/gaps_c$c.json
done
