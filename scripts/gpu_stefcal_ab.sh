#!/bin/bash
# StefCal A/B: solver parity (irregular-CSR test on the reference build, all
# solver tests on the in-tree build), then the stefcal path timing for each
# library given (exp/<name>.so, or "tree").
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/stef; mkdir -p $out
SDP_HIP_LIB_OVERRIDE=$PWD/exp/stef_old.so timeout -k 10 200 python -u -m pytest tests/test_gpu_solvers.py -x -q -k irregular --timeout 120 --timeout-method thread -p no:cacheprovider > $out/old.log 2>&1
rc=$?; echo "old-lib irregular rc=$rc"; tail -2 $out/old.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_parallel.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/new.log 2>&1
rc=$?; echo "tree solvers rc=$rc"; tail -2 $out/new.log
[ $rc -ne 0 ] && exit $rc
for v in "$@"; do
  if [ $v = tree ]; then unset SDP_HIP_LIB_OVERRIDE; else export SDP_HIP_LIB_OVERRIDE=$PWD/exp/$v.so; fi
  timeout -k 10 120 python scripts/bench_paths.py stefcal 2>&1 | grep '^{' | sed "s/^/$v /" || exit 1
done
