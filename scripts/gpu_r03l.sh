#!/bin/bash
# r03l: C2 invert A/B (in-tree HEAD build vs abvar/gpre.so: the gridder's
# first record load above the region zeroing + the degridder's branchless
# stores), C2 predict A/B (same pair), then the NUFFT parity tests on gpre
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
R=2 bash scripts/gpu_ab.sh cur abvar/gpre.so || exit 1
for r in 1 2; do
  timeout -k 10 200 python scripts/predict_time.py || exit 1
  SDP_HIP_LIB_OVERRIDE=abvar/gpre.so timeout -k 10 200 python scripts/predict_time.py || exit 1
done
SDP_HIP_LIB_OVERRIDE=abvar/gpre.so timeout -k 10 600 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_fullsize.py tests/test_gpu_orientation.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03l_pytest.log 2>&1 || { tail -30 gpurun_out/r03l_pytest.log; exit 1; }
tail -1 gpurun_out/r03l_pytest.log
