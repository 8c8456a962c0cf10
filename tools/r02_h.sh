set -o pipefail
out=gpurun_out/r02_h; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "lanes or walk or config3 or hot_limits" > $out/tests.log 2>&1; rc=$?; tail -25 $out/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_configs.py --configs 3 > $out/configs.json 2> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
cat $out/configs.json
