set -o pipefail
tag=${1:-r02_bench}; shift
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py "$@" > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r['path']['frac'],r['kernels_ms_per_step'])"
