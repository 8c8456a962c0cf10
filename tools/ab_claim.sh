set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_claim_tests.log 2>&1 || exit 1
for v in default prev default prev; do
  lib=""; [ "$v" = default ] || lib=$PWD/tigerbeetle_amd/lib/variants/libtbg_$v.so
  for a in wide exp; do
    TBG_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --configs 3,4 --amounts $a > gpurun_out/r05_claim_${v}_$a.json 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/r05_claim_${v}_$a.json'):
    if l.startswith('{'): d=json.loads(l); print('$v $a', d['config'], d['device_transfers_per_s'], d['gpu_transfers_per_s'], d['kernels_ms'].get('account_events'))
"
  done
done
