#!/bin/bash
# C2 predict A/B: the in-tree build against abvar/$1.so, alternated twice,
# then the predict parity tests on the variant.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
v=$1
for r in 1 2; do
  timeout -k 10 200 python scripts/predict_time.py || exit 1
  SDP_HIP_LIB_OVERRIDE=abvar/$v.so timeout -k 10 200 python scripts/predict_time.py || exit 1
done
SDP_HIP_LIB_OVERRIDE=abvar/$v.so timeout -k 10 500 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_fullsize.py::test_c2_full_predict_against_reference_precision tests/test_gpu_skymodel.py tests/test_gpu_orientation.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "dirty2ms or predict or adjoint or round_trip or skymodel or orientation or unit_pixel" > gpurun_out/${v}_predict_pytest.log 2>&1 || { tail -30 gpurun_out/${v}_predict_pytest.log; exit 1; }
tail -1 gpurun_out/${v}_predict_pytest.log
