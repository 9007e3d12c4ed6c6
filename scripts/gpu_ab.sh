#!/bin/bash
# A/B of library builds on the C2 bench step: alternates the builds given as
# arguments (paths to libska_sdp_hip.so variants; "cur" = the in-tree build)
# R times, printing each run's step time and stage breakdown.
cd "$(dirname "$0")/.." || exit 1
R=${R:-2}
for r in $(seq 1 $R); do
  for lib in "$@"; do
    if [ "$lib" = cur ]; then unset SDP_HIP_LIB_OVERRIDE; else export SDP_HIP_LIB_OVERRIDE=$lib; fi
    out=$(timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extra --no-api --cpu-chans 0 2>/dev/null) || { echo "FAILED $lib"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib', d['value'], d['ms_per_step'], d['stages_ms'], d['roofline']['kernel_ms'])"
  done
done
