mkdir -p gpurun_out/lanes1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lanes1/tests.log 2>&1 || { tail -30 gpurun_out/lanes1/tests.log; exit 1; }
tail -2 gpurun_out/lanes1/tests.log
timeout -k 10 300 python -u tools/bench_configs.py --transfers 1000000 > gpurun_out/lanes1/configs.json 2> gpurun_out/lanes1/err.log || { tail gpurun_out/lanes1/err.log; exit 1; }
cat gpurun_out/lanes1/configs.json
