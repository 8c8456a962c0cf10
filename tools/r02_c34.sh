set -o pipefail
tag=${1:-r02_c34}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_configs.py --configs 3,4 > $out/configs.json 2> $out/configs.err || { tail -20 $out/configs.err; exit 1; }
cat $out/configs.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs 3,4 > $GRAFT_REPO_ROOT/$out/prof_configs.json 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
cut -d, -f1-4 $out/kernel_stats.csv | cut -c1-140 | head -30
