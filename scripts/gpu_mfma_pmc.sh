#!/bin/bash
# SQ PMC passes on the invert gridding kernel (C2), one counter set per pass.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-pmc_mfma}
mkdir -p $out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_INSTS_BRANCH" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "${KRX:-k_grid}" --output-format csv -d $out/p$i -o run -- \
      python3 scripts/gpu_sweep.py SDP_HIP_DBG ${DBG:-0} > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; }
done
python3 - "$out" <<'PY'
import csv, collections, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/run_counter_collection.csv", recursive=True) + glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    if not rows:
        continue
    last = max(int(r["Dispatch_Id"]) for r in rows)
    d = collections.defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            d[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f, rows[0]["Kernel_Name"][:40], {k: int(v) for k, v in d.items()})
PY
