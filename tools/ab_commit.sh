# Same-box A/B of library variants on the per-commit path (tools/commit_timeline.py, no profiling):
# bash tools/ab_commit.sh <tag> <variant>... ("default" = tigerbeetle_amd/lib/libtbg.so, else
# tigerbeetle_amd/lib/variants/libtbg_<variant>.so). Three alternating rounds of 300 commits.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
for round in 1 2 3; do
  for v in "$@"; do
    if [ "$v" = default ]; then lib=""; else lib=$PWD/tigerbeetle_amd/lib/variants/libtbg_$v.so; fi
    TBG_LIB=$lib timeout -k 10 120 python -u tools/commit_timeline.py --commits 300 --mode 0 > $out/commit_$v.$round.json 2> $out/commit_$v.$round.err || { tail -5 $out/commit_$v.$round.err; exit 1; }
    echo "$v $round $(cut -c1-300 $out/commit_$v.$round.json)"
  done
done
