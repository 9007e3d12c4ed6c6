#!/bin/bash
# r03c extras: C2 predict timing of the in-tree build against abvar/head.so
# (alternated), then the C4 N = 1 PMC passes
cd "$(dirname "$0")/.." || exit 1
for r in 1 2; do
  timeout -k 10 200 python scripts/predict_time.py || exit 1
  SDP_HIP_LIB_OVERRIDE=abvar/head.so timeout -k 10 200 python scripts/predict_time.py || exit 1
done
bash scripts/pmc_c4.sh r03c || exit $?
