#!/bin/bash
# compact fp64 records: f64 tests, then A/B vs HEAD lib (C2 eps 1e-12)
cd "$(dirname "$0")/.." || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nufft_f64.py tests/test_gpu_skymodel.py > gpurun_out/f64_tests.log 2>&1; rc=$?; tail -3 gpurun_out/f64_tests.log; [ $rc -eq 0 ] || exit $rc
for L in abtmp/lib_head.so "" abtmp/lib_head.so ""; do
  echo "== lib ${L:-in-tree}"
  SDP_HIP_LIB_OVERRIDE=$L timeout -k 10 200 python3 scripts/time_c2.py --reps 3 --eps 1e-12 || exit 1
done
