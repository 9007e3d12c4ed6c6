#!/bin/bash
# streamed host-Visibility invert: tests + api timing
cd "$(dirname "$0")/.." || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nufft.py -k "host_visibility_streamed or fused_prologue or batched or cube_channel" > gpurun_out/host_tests.log 2>&1; rc=$?; tail -3 gpurun_out/host_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_skymodel.py > gpurun_out/sky_tests.log 2>&1; rc=$?; tail -3 gpurun_out/sky_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 4 1 8 4; do
  echo "== host blocks $b"
  SDP_HIP_HOST_BLOCKS=$b timeout -k 10 300 python3 bench.py --no-extra --cpu-chans 0 --steps 2 > gpurun_out/api_$b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/api_$b.json').read().strip().splitlines()[-1]); a=d['api']; print(a['invert_ng_host_visibility_ms'], a['invert_ng_device_visibility_ms'])"
done
