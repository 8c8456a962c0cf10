set -o pipefail
out=gpurun_out/r02_q; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tables.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "table or fuzz or scans" > $out/tests.log 2>&1; rc=$?; tail -30 $out/tests.log; exit $rc
