#!/bin/bash
# Instruction mix of the flow replay on one lane (config 4): SQ counters per flow_replay dispatch.
set -o pipefail
tag=${1:-flowpmc}; out=$GRAFT_REPO_ROOT/gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp TBG_FLOW_LPW=1 TBG_FLOW_WAVES=1 TBG_FLOW_BLOCKS=1
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH \
  --output-format csv -d $out/pmc -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs 4 > $out/run.json 2> $out/run.err || { tail -5 $out/run.err; exit 1; }
f=$(find $out/pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
agg=collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if 'flow_replay' not in r['Kernel_Name']: continue
    agg[r['Dispatch_Id']][r['Counter_Name']]+=float(r['Counter_Value'])
for d,v in sorted(agg.items(), key=lambda x:int(x[0])):
    print(d, {k:int(x) for k,x in sorted(v.items())})
PY
