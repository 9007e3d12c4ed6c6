#!/bin/bash
# C4 strong scaling on one GPU: the full 256-channel band on 1 GPU (bench.py
# --config c4), then every rank of the 2-, 4- and 8-way cost-balanced
# partitions emulated one at a time (per-rank step times, no collective).
# C4ARGS: extra bench.py arguments (C4N1ARGS for the N = 1 run, default C4ARGS);
# WORLDS: the partitions (default 8 4 2).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
tag=${1:-r02}
out=gpurun_out/${tag}_c4_scaling.jsonl
: > $out
timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 ${C4N1ARGS-$C4ARGS} > gpurun_out/${tag}_c4_n1.log 2>&1 || exit $?
grep '^{' gpurun_out/${tag}_c4_n1.log >> $out
for w in ${WORLDS:-8 4 2}; do
  for ((r = 0; r < w; r++)); do
    timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 ${C4ARGS} --emulate $r/$w > gpurun_out/${tag}_c4_e${r}_${w}.log 2>&1 || exit $?
    grep '^{' gpurun_out/${tag}_c4_e${r}_${w}.log >> $out
  done
done
cat $out
