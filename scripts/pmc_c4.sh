#!/bin/bash
# C4 N = 1 (bench.py --config c4): rocprofv3 kernel stats, then FETCH_SIZE and
# WRITE_SIZE of the gridding launches in separate --pmc passes (MI355X_MICROARCH.md
# HBM section), summed over the batch launches of the last invert ->
# gpurun_out/<tag>_c4/traffic_c4_k_grid.json (copy to profiles/ for bench.py)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tag=${1:-r03}
out=gpurun_out/${tag}_c4
mkdir -p $out
args="--config c4 --steps 1 --warmup 0 --c4-cpu-chans 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 bench.py $args > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- \
      python3 bench.py $args > $out/$c.log 2>&1 || { tail -20 $out/$c.log; exit 1; }
done
python3 scripts/summarize_c4_pmc.py $out
