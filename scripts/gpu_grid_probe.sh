#!/bin/bash
# Gridder ablations (SDP_HIP_DBG knobs) + one SQ PMC pass on k_grid_reg.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-probe}
mkdir -p $out
timeout -k 10 300 python scripts/gpu_sweep.py SDP_HIP_DBG 0,1,2,4 > $out/sweep.log 2>&1 || { tail -20 $out/sweep.log; exit 1; }
grep -v amdgpu.ids $out/sweep.log
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
   --kernel-include-regex "k_grid" --output-format csv -d $out/p1 -o run -- python3 scripts/gpu_sweep.py SDP_HIP_DBG 0 > $out/p1.log 2>&1 || { tail -20 $out/p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
   --kernel-include-regex "k_grid" --output-format csv -d $out/p2 -o run -- python3 scripts/gpu_sweep.py SDP_HIP_DBG 0 > $out/p2.log 2>&1 || { tail -20 $out/p2.log; exit 1; }
find $out -name "*counter_collection.csv"
