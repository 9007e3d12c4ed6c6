#!/bin/bash
# Predict parity, then the C2 predict path with SDP_HIP_ZERO_OVERLAP on / off (alternating).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_fullsize.py::test_c2_full_predict_against_reference_precision tests/test_gpu_skymodel.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "dirty2ms or predict or adjoint or round_trip or skymodel" > gpurun_out/pz_pytest.log 2>&1 || { tail -30 gpurun_out/pz_pytest.log; exit 1; }
tail -1 gpurun_out/pz_pytest.log
for rep in 1 2; do
  for z in 1 0; do
    echo "== SDP_HIP_ZERO_OVERLAP=$z"
    SDP_HIP_ZERO_OVERLAP=$z timeout -k 10 200 python scripts/bench_paths.py predict 2>&1 | grep '^{' | cut -c1-240 || exit 1
  done
done
