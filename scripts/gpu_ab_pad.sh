#!/bin/bash
# Parity of the tree build's invert path, then C2 stage timings of kernel variants (exp/*.so).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_fullsize.py::test_c2_full_invert_against_reference_precision -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
for v in tree "$@"; do
  if [ $v = tree ]; then unset SDP_HIP_LIB_OVERRIDE; else export SDP_HIP_LIB_OVERRIDE=$PWD/exp/$v.so; fi
  echo "== $v"
  timeout -k 10 200 python scripts/gpu_sweep.py SDP_HIP_DUMMY 0,1 2>&1 | grep -v amdgpu.ids || exit 1
done
