# Same-box A/B of library variants on config 2's AccountEvents (Exp and wide amounts):
# bash tools/ab_ae.sh <tag> <variant>... ("default" = libtbg.so, else
# tigerbeetle_amd/lib/variants/libtbg_<variant>.so). Prints the appends' ms per 10M-event step.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
for round in 1 2; do
  for amounts in exp wide; do
    for v in "$@"; do
      if [ "$v" = default ]; then lib=""; else lib=$PWD/tigerbeetle_amd/lib/variants/libtbg_$v.so; fi
      TBG_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --commit-reps 0 --no-hazard-call --steps 3 --amounts $amounts > $out/$v.$amounts.$round.json 2> $out/$v.$amounts.$round.err || { tail -5 $out/$v.$amounts.$round.err; exit 1; }
      python -c "import json;d=json.load(open('$out/$v.$amounts.$round.json'));a=d['with_account_events'];print('$v', '$amounts', $round, a['account_events_ms_per_step'], a['ms_per_step'], d['ms_per_step'])"
    done
  done
done
