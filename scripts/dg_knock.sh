#!/bin/bash
# knock-out: predict without the output zeroing (C2 has no unbucketed visibility)
cd "$(dirname "$0")/.." || exit 1
for z in 0 1 0 1; do
  echo "== skip $z"
  SDP_HIP_ZV_SKIP=$z timeout -k 10 200 python3 scripts/time_c2.py --reps 7 || exit 1
done
