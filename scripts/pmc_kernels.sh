#!/bin/bash
# PMC passes (one counter set per rocprofv3 run) over the kernels matching a
# regex while a command runs, plus a kernel trace; per-kernel sums printed
# (all launches of each kernel in the run).
#   scripts/pmc_kernels.sh <tag> <kernel-regex> <command ...>
# e.g. scripts/pmc_kernels.sh f64 "k_grid_f64|k_degrid_f64" python3 scripts/time_c2.py --reps 1 --eps 1e-12
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tag=$1; rx=$2; shift 2
out=gpurun_out/pmc_${tag}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    "$@" > $out/trace.log 2>&1 || { echo "trace failed"; tail -20 $out/trace.log; exit 1; }
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --kernel-include-regex "$rx" --output-format csv -d $out/p$i -o run -- \
      "$@" > $out/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -5 $out/p$i.log; }
done
python3 - "$out" <<'PY'
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
