#!/bin/bash
# PMC counters of one kernel (default: the gridder) on the C2 workload, one
# rocprofv3 --pmc pass per counter set (no trace domains), then a JSON
# summary of the last dispatch: scripts/pmc_grid.sh TAG [KERNEL_REGEX] [--predict]
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tag=${1:-pmc}
kre=${2:-k_grid}
shift 2 2>/dev/null
out=gpurun_out/$tag
mkdir -p $out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32" \
           "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$kre" --output-format csv -d $out/p$i -o run -- \
      python3 scripts/grid_once.py "$@" > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $out/p$i.log; exit 1; }
done
python3 - $out "$kre" <<'PY'
import csv, glob, json, os, sys
out, kre = sys.argv[1], sys.argv[2]
res = {}
for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    rows = list(csv.DictReader(open(f)))
    last = max(int(r["Dispatch_Id"]) for r in rows)
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            res[r["Counter_Name"]] = res.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            res["kernel"] = r["Kernel_Name"][:90]
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(out, "pmc.json"), "w"), indent=1)
PY
