#!/bin/bash
# C2 headline pipelined with stream CU-mask variants
cd "$(dirname "$0")/.." || exit 1
for m in alt ovl "" alt ovl ""; do
  echo "== cu-split '$m'"
  timeout -k 10 300 python3 bench.py --no-extra --no-api --cpu-chans 0 --steps 10 --cu-split "$m" || exit 1
done
