#!/bin/bash
# PMC passes over configs 3 / 4 (tools/bench_configs.py, no HIP-event marks), one counter group per
# rocprofv3 run; summarised per kernel by tools/pmc_summary.py.
# Usage (repo root, via gpurun): bash tools/pmc_c34.sh <tag> [bench_configs args...]
set -o pipefail
tag=${1:-pmc_c34}; shift
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
args="--no-profile $*"
i=0
passes=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
        "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
        "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCC_ATOMIC_sum")
for ctrs in "${passes[@]}"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $ctrs --output-format csv -d $out/p$i -o run -- \
        python3 $R/tools/bench_configs.py $args > $out/p$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -5 $out/p$i.log; exit 1; }
done
cd $R && python3 tools/pmc_summary.py $out $out/traffic.json > $out/summary.txt && echo ok
