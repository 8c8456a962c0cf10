# Same-box A/B of library variants on the wide-amount AccountEvents kernels (ae_wide_*): config 2's
# step with the account_events groove under --amounts wide, one kernel trace per variant.
# bash tools/ab_wide_ae.sh <tag> <variant>... ("default" = libtbg.so; AMOUNTS=exp for the narrow window)
set -o pipefail
tag=$1; shift
out=$PWD/gpurun_out/$tag; mkdir -p $out
repo=$PWD
for v in "$@"; do
  lib=""
  [ "$v" = default ] || lib=$repo/tigerbeetle_amd/lib/variants/libtbg_$v.so
  (cd /tmp && export TMPDIR=/tmp && TBG_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace_$v -o run -- python3 $repo/bench.py --amounts ${AMOUNTS:-wide} --no-cpu-baseline --steps 2 --warmup 1 --commit-reps 10 --no-routed > $out/bench_$v.json 2> $out/bench_$v.err) || { tail -5 $out/bench_$v.err; exit 1; }
  python3 - "$out/trace_$v" "$v" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "ae_wide" in n or "ae_window" in n:
        d[n.split("(")[0].replace("tbg::", "")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(sys.argv[2], {k: round(sum(v) / len(v), 1) for k, v in d.items()})
PY
done
