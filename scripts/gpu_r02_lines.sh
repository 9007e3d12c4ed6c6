#!/bin/bash
# C3 / C5 bench lines, predict path line, C2 kernel statistics (each step time-limited).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 > gpurun_out/c3_bench.log 2>&1 || exit $?
tail -1 gpurun_out/c3_bench.log
timeout -k 10 400 python bench.py --config c5 --steps 1 --warmup 0 > gpurun_out/c5_bench.log 2>&1 || exit $?
tail -1 gpurun_out/c5_bench.log
timeout -k 10 300 python scripts/bench_paths.py predict > gpurun_out/predict_path.log 2>&1 || exit $?
tail -1 gpurun_out/predict_path.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o c2 -- python bench.py --steps 5 --warmup 2 --cpu-chans 0 --no-api > gpurun_out/c2_prof_bench.log 2>&1 || exit $?
tail -1 gpurun_out/c2_prof_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 -- python bench.py --config c3 --steps 10 --warmup 2 > gpurun_out/c3_prof_bench.log 2>&1 || exit $?
find gpurun_out/prof_c2 gpurun_out/prof_c3 -name "*stats*"
