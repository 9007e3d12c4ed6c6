#!/bin/bash
# PMC counter sets, one rocprofv3 --pmc run per set, over the kernels matching
# a regex while a command runs (plus one kernel trace); per-kernel sums of
# every launch printed and written to gpurun_out/pmc_<tag>/summary.txt.
#   scripts/pmc_sets.sh <tag> <kernel-regex> "<set1>" ["<set2>" ...] -- <command ...>
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tag=$1; rx=$2; shift 2
sets=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do sets+=("$1"); shift; done
shift
out=gpurun_out/pmc_${tag}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "$rx" --output-format csv \
    -d $out/trace -o run -- "$@" > $out/trace.log 2>&1 || { echo "trace failed"; tail -20 $out/trace.log; exit 1; }
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --kernel-include-regex "$rx" --output-format csv -d $out/p$i -o run -- \
      "$@" > $out/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -3 $out/p$i.log; }
done
python3 - "$out" > $out/summary.txt <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
for f in sorted(glob.glob(out + "/trace/**/*kernel_stats.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        print("stats", r["Name"].split("(")[0][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(f)))
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"].split("(")[0][:60]
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
    for k, v in d.items():
        print(f.split("/")[len(out.split("/"))], k, "launches", len(n[k]), {c: int(x) for c, x in v.items()})
PY
cat $out/summary.txt
