#!/bin/bash
# PMC passes over a short bench run, one counter group per rocprofv3 run (MI355X_MICROARCH.md
# "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Usage (repo root, via gpurun): bash tools/pmc.sh <tag> [bench args...]
set -o pipefail
tag=${1:-pmc}; shift
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
args="--no-cpu-baseline --no-validate --commit-reps 0 --steps 2 --warmup 1 $*"
i=0
# PMC_TRAFFIC_ONLY=1: the two HBM traffic passes only (what roofline.traffic reads).
passes=("FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
            "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
            "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
            "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCC_ATOMIC_sum")
[ -n "$PMC_TRAFFIC_ONLY" ] && passes=("FETCH_SIZE" "WRITE_SIZE")
for ctrs in "${passes[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $out/p$i -o run -- \
        python3 $R/bench.py $args > $out/p$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -5 $out/p$i.log; exit 1; }
done
cd $R && python3 tools/pmc_summary.py $out $out/traffic.json > $out/summary.txt && cat $out/traffic.json
# (the per-launch averages cover only full-size bench steps: --commit-reps 0 runs no 8189-event
# per-commit calls, whose launches would otherwise be averaged in)
