#!/bin/bash
# A/B of library variants on the C2 invert and predict (scripts/time_c2.py);
# arguments as scripts/gpu_ab.sh (LIB[,VAR=VAL...], "cur" = in-tree build)
cd "$(dirname "$0")/.." || exit 1
R=${R:-2}
for r in $(seq 1 $R); do
  for spec in "$@"; do
    IFS=',' read -ra parts <<< "$spec"
    lib=${parts[0]}
    envs=("${parts[@]:1}")
    if [ "$lib" = cur ]; then L=""; else L="SDP_HIP_LIB_OVERRIDE=$lib"; fi
    out=$(env $L "${envs[@]}" timeout -k 10 200 python3 scripts/time_c2.py 2>/dev/null) || { echo "FAILED $spec"; exit 1; }
    echo "$spec $(echo "$out" | tail -1)"
  done
done
