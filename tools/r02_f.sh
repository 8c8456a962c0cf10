set -o pipefail
out=gpurun_out/r02_f; mkdir -p $out
timeout -k 10 400 python -u bench.py --commit-reps 50 > $out/bench.json 2> $out/bench.err && cat $out/bench.json &&
TBG_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --transfers 2000000 --routed-transfers 500000 > $out/bench2.json 2> $out/bench2.err && cat $out/bench2.json
