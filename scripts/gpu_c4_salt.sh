#!/bin/bash
# C4 N = 1 with the coarse-bucket salt (SDP_HIP_SALT) at 1, 2 and 4: the count
# pass's counters are ntiles x nps x salt x 4 B (salt 1: ~250 MB, inside the
# 256 MB MALL, where returning atomics run at 27 G/s instead of 19 G/s)
cd "$(dirname "$0")/.." || exit 1
for s in 1 2 4 1 2 4; do
  out=$(SDP_HIP_SALT=$s timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 --c4-cpu-chans 0 2>/dev/null | grep '^{') || { echo "FAILED salt $s"; exit 1; }
  echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('salt $s', d['value'], d['ms_per_step'], d['stages_ms_rank0'])"
done
