# Same-box A/B of library variants: bash tools/ab_bench.sh <tag> <variant>... (variant "default"
# = tigerbeetle_amd/lib/libtbg.so, else tigerbeetle_amd/lib/variants/libtbg_<variant>.so)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then lib=""; else lib=$PWD/tigerbeetle_amd/lib/variants/libtbg_$v.so; fi
    TBG_LIB=$lib timeout -k 10 200 python -u bench.py --no-validate --no-cpu-baseline --commit-reps 0 --steps 10 > $out/$v.$round.json 2> $out/$v.$round.err || { tail -5 $out/$v.$round.err; exit 1; }
    python -c "import json;d=json.load(open('$out/$v.$round.json'));r=d['roofline'];print('$v', $round, d['value'],d['ms_per_step'],r['avg_launch_ms'],r['kernels_ms_per_step'])"
  done
done
