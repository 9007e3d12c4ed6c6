#!/bin/bash
# SQ PMC passes (one rocprofv3 run per counter set) plus a kernel-trace stats
# run, on the kernels matching a regex, for any python probe.
# usage: gpu_pmc.sh tag kernel_regex script.py [args]
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/$1; kre=$2; shift 2
mkdir -p $out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex "$kre" --output-format csv -d $out/p$i -o run -- \
      python3 "$@" > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $out/p$i.log; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 "$@" > $out/kt.log 2>&1 || exit 1
python3 - "$out" "$kre" <<'PY'
import csv, collections, glob, re, sys
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    rows = [r for r in csv.DictReader(open(f)) if re.search(sys.argv[2], r["Kernel_Name"])]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    d = collections.defaultdict(float)
    for r in rows:
        d[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f.split("/")[-2], rows[0]["Kernel_Name"][:30], "dispatches", len(ids),
          {k: round(v / len(ids)) for k, v in d.items()})
for f in glob.glob(sys.argv[1] + "/kt/run_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print("stats", r["Name"][:50], r["Calls"], "avg ns", r["AverageNs"], "pct", r.get("Percentage"))
PY
