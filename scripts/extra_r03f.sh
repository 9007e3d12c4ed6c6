#!/bin/bash
# r03f extras: C2 predict timing in-tree (batched region loads in the
# degridder) vs abvar/head2.so (alternated), then the C4 channel-block 8-way
# emulation with the refitted cost model
cd "$(dirname "$0")/.." || exit 1
for r in 1 2; do
  timeout -k 10 200 python scripts/predict_time.py || exit 1
  SDP_HIP_LIB_OVERRIDE=abvar/head2.so timeout -k 10 200 python scripts/predict_time.py || exit 1
done
WORLDS=8 C4ARGS="--partition chan" bash scripts/gpu_c4_scaling.sh r03f > gpurun_out/r03f_c4.log 2>&1 || { tail -20 gpurun_out/r03f_c4.log; exit 1; }
python3 scripts/c4_scaling_summary.py gpurun_out/r03f_c4_scaling.jsonl
