#!/bin/bash
# C4 per-rank stage times for the 8 contiguous channel blocks of the
# 256-channel SKA-LOW band (one GPU, one block at a time).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
out=gpurun_out/${1:-r02}_c4_blocks.jsonl
: > $out
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 240 python -u scripts/bench_c4_shard.py --layout block --rank $r --reps 2 > gpurun_out/c4_block_$r.log 2>&1 || exit $?
  grep '^{' gpurun_out/c4_block_$r.log >> $out
done
cat $out
