#!/bin/bash
# PMC passes on the two-level bucketing kernels of the C2 invert
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/pmc_tb
mkdir -p $out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "k_t_" --output-format csv -d $out/p$i -o run -- \
      python3 scripts/time_c2.py --reps 1 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $out/p$i.log; exit 1; }
done
python3 - "$out" <<'PY'
import csv, collections, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in rows:
        k = r["Kernel_Name"].split("(")[0][:60]
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in d.items():
        print(f.split("/")[-2], k, {c: int(x) for c, x in v.items()})
PY
