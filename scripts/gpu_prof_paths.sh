#!/bin/bash
# rocprofv3 kernel statistics of the predict path (C2) and of a C5 slice.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pred -o pred -- python3 scripts/bench_paths.py predict > gpurun_out/prof_pred.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_pred.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o c5 -- python3 bench.py --config c5 --c5-times 96 --steps 1 --warmup 1 > gpurun_out/prof_c5.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_c5.log | cut -c1-200
find gpurun_out/prof_pred gpurun_out/prof_c5 -name "*kernel_stats.csv"
