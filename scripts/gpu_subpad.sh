#!/bin/bash
# Parity of the sub-sorted padded invert path (large grids), then C4 rank
# blocks and the whole band with SDP_HIP_SUBSORT_PAD on / off.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_fullsize.py::test_c4_shard_invert_predict_at_full_size -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/subpad_pytest.log 2>&1 || { tail -40 gpurun_out/subpad_pytest.log; exit 1; }
tail -1 gpurun_out/subpad_pytest.log
for pad in 1 0; do
  echo "== SDP_HIP_SUBSORT_PAD=$pad"
  for r in 7 0 3; do
    SDP_HIP_SUBSORT_PAD=$pad timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --emulate $r/8 2>&1 | grep '^{' || exit 1
  done
done
timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 > gpurun_out/subpad_c4_n1.log 2>&1 || exit 1
grep '^{' gpurun_out/subpad_c4_n1.log | cut -c1-200
grep -o '"stages_ms_rank0": {[^}]*}' gpurun_out/subpad_c4_n1.log
