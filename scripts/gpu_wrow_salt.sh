#!/bin/bash
# Row-partition ranks whose rows are the dense uv core (4-way ranks 1, 2; 8-way
# rank 5) at coarse-bucket salt 4 / 16 / 32: their count pass is bound by the
# serial atomics on the hot buckets' counters
cd "$(dirname "$0")/.." || exit 1
for spec in "1/4 4" "1/4 16" "1/4 32" "5/8 4" "5/8 16" "5/8 32"; do
  set -- $spec
  out=$(SDP_HIP_SALT=$2 timeout -k 10 300 python bench.py --config c4 --partition wrow --emulate $1 --steps 2 --warmup 1 2>/dev/null | grep '^{') || { echo "FAILED $spec"; exit 1; }
  echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rank $1 salt $2', d['ms_per_step'], {k: round(v, 1) for k, v in d['stages_ms'].items()})"
done
