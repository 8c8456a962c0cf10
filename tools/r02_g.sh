set -o pipefail
out=gpurun_out/r02_g; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_durability.py -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -30 $out/tests.log; exit $rc
