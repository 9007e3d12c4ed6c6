#!/bin/bash
# A/B of library builds / knobs on the C2 bench step.  Each argument is
# LIB[,VAR=VAL...]: LIB a libska_sdp_hip.so variant path or "cur" (the
# in-tree build), followed by environment settings for that run.  The
# variants are alternated R times; each run prints its step time and stages.
cd "$(dirname "$0")/.." || exit 1
R=${R:-2}
for r in $(seq 1 $R); do
  for spec in "$@"; do
    IFS=',' read -ra parts <<< "$spec"
    lib=${parts[0]}
    envs=("${parts[@]:1}")
    if [ "$lib" = cur ]; then L=""; else L="SDP_HIP_LIB_OVERRIDE=$lib"; fi
    out=$(env $L "${envs[@]}" timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extra --no-api --cpu-chans 0 2>/dev/null) || { echo "FAILED $spec"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$spec', d['value'], d['ms_per_step'], d['stages_ms'], d['roofline']['kernel_ms'])"
  done
done
