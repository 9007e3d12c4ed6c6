#!/bin/bash
# C2 stage timings, alternating the tree build and variants (exp/*.so), twice.
cd "$(dirname "$0")/.." || exit 1
for rep in 1 2; do
  for v in tree "$@"; do
    if [ $v = tree ]; then unset SDP_HIP_LIB_OVERRIDE; else export SDP_HIP_LIB_OVERRIDE=$PWD/exp/$v.so; fi
    echo "== $v"
    timeout -k 10 200 python scripts/gpu_sweep.py SDP_HIP_DUMMY 0,1 2>&1 | grep '^{' || exit 1
  done
done
