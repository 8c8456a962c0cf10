# Same-box A/B on the per-commit path (tools/commit_timeline.py, no profiling):
# bash tools/ab_commit.sh <tag> <variant>... -- "default" = tigerbeetle_amd/lib/libtbg.so;
# "env:NAME" = the default library with NAME=1 in the environment; else
# tigerbeetle_amd/lib/variants/libtbg_<variant>.so. Three alternating rounds of 300 commits.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
for round in 1 2 3; do
  for v in "$@"; do
    lib=""; envs=""
    case $v in
      default) ;;
      env:*) envs="${v#env:}=1" ;;
      *) lib=$PWD/tigerbeetle_amd/lib/variants/libtbg_$v.so ;;
    esac
    f=$(echo "$v" | tr ':' '_')
    env TBG_LIB=$lib $envs timeout -k 10 120 python -u tools/commit_timeline.py --commits 300 --mode 0 > $out/commit_$f.$round.json 2> $out/commit_$f.$round.err || { tail -5 $out/commit_$f.$round.err; exit 1; }
    echo "$v $round $(cut -c1-200 $out/commit_$f.$round.json)"
  done
done
