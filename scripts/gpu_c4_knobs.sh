#!/bin/bash
# C4 N = 1 knob sweep (bench.py --config c4, 1 warmup + 2 steps each):
# coarse-bucket salt (SDP_HIP_SALT) and the visibilities per streamed batch
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for spec in ${C4SPECS:-"SDP_HIP_SALT=4 1.8" "SDP_HIP_SALT=8 1.8" "SDP_HIP_SALT=16 1.8"}; do
  set -- $spec
  out=$(env $1 timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 --c4-cpu-chans 0 --c4-batch-gvis $2 2>/dev/null | grep '^{') || { echo "FAILED $spec"; exit 1; }
  echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', d['value'], d['ms_per_step'], d['config']['rank0_batches'], d['stages_ms_rank0'])"
done
