#!/bin/bash
# PMC counters for the gridding kernel (separate passes, kernel filter)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp SDP_HIP_GRID_WAVES=${WAVES:-2}
tag=${1:-pmc}
out=gpurun_out/$tag
mkdir -p $out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "k_grid" --output-format csv -d $out/p$i -o run -- \
      python3 scripts/gpu_sweep.py SDP_HIP_BUCKET ${BUCKET:-2} > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $out/p$i.log; exit 1; }
done
find $out -name "*counter_collection.csv"
