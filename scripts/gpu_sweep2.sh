#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
for order in 1 0; do
  for waves in 1 4; do
    export SDP_HIP_ITEM_ORDER=$order SDP_HIP_GRID_WAVES=$waves
    echo "order=$order waves=$waves"
    timeout -k 10 300 python scripts/gpu_sweep.py SDP_HIP_CHUNK 2048,7544,16384 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
