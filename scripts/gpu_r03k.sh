#!/bin/bash
# r03k: the slot / stream overlap test first, then the full GPU suite and
# smoke, then C2 bench steps pipelined vs serial (alternated), then the
# default bench line
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_nufft.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "two_slots" > gpurun_out/r03k_slots.log 2>&1 || { tail -30 gpurun_out/r03k_slots.log; exit 1; }
tail -1 gpurun_out/r03k_slots.log
for r in 1 2; do
  for m in "" "--no-pipeline"; do
    out=$(timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extra --no-api --cpu-chans 0 $m 2>/dev/null | grep '^{') || { echo "FAILED bench $m"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pipe' if '$m' == '' else 'serial', d['value'], d['ms_per_step'], d['config']['ms_per_step_serial'], d['roofline']['kernel_ms'])"
  done
done
bash scripts/gpu_session.sh r03k
