#!/bin/bash
# r03d extras: C2 predict timing in-tree vs abvar/prev.so (alternated), then
# the C4 scaling emulation: N = 1 and the 8 ranks of the 8-way w-slab partition
cd "$(dirname "$0")/.." || exit 1
for r in 1 2; do
  timeout -k 10 200 python scripts/predict_time.py || exit 1
  SDP_HIP_LIB_OVERRIDE=abvar/prev.so timeout -k 10 200 python scripts/predict_time.py || exit 1
done
WORLDS=8 C4ARGS="--partition wslab" bash scripts/gpu_c4_scaling.sh r03d || exit $?
python3 scripts/c4_scaling_summary.py gpurun_out/r03d_c4_scaling.jsonl
