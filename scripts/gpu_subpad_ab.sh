#!/bin/bash
# C4 rank blocks (8-way partition) with SDP_HIP_SUBSORT_PAD on / off, alternating.
cd "$(dirname "$0")/.." || exit 1
for r in 7 0 3; do
  for pad in 1 0; do
    echo "== rank $r/8 SDP_HIP_SUBSORT_PAD=$pad"
    SDP_HIP_SUBSORT_PAD=$pad timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --emulate $r/8 2>&1 | grep '^{' || exit 1
  done
done
