# Same-box A/B of library variants on bench.py's per-commit lines (device and StateMachine):
# bash tools/ab_percommit.sh <tag> <variant>... ("default" = libtbg.so, else
# tigerbeetle_amd/lib/variants/libtbg_<variant>.so). Three alternating rounds.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
for round in 1 2 3; do
  for v in "$@"; do
    lib=""
    [ "$v" = default ] || lib=$PWD/tigerbeetle_amd/lib/variants/libtbg_$v.so
    TBG_LIB=$lib timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-account-events-line --commit-reps 300 > $out/pc_$v.$round.json 2> $out/pc_$v.$round.err || { tail -5 $out/pc_$v.$round.err; exit 1; }
    python3 -c "import json;d=json.load(open('$out/pc_$v.$round.json'))['per_commit'];print('$v', $round, 'device', d['device']['us_per_commit_mean'], d['device']['us_per_commit_p50'], 'sm', d['state_machine']['us_per_commit_mean'], d['state_machine']['us_per_commit_p50'])"
  done
done
