#!/bin/bash
# A/B: 32- (in-tree) vs 48-record fp64 gridder blocks, C2 eps 1e-12
cd "$(dirname "$0")/.." || exit 1
for L in "" abtmp/lib_blk48.so "" abtmp/lib_blk48.so; do
  echo "== lib ${L:-in-tree}"
  SDP_HIP_LIB_OVERRIDE=$L timeout -k 10 200 python3 scripts/time_c2.py --reps 3 --eps 1e-12 || exit 1
done
