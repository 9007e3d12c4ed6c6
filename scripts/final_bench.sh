#!/bin/bash
# the default bench line on the current build -> gpurun_out/bench_final.json
cd "$(dirname "$0")/.." || exit 1
timeout -k 10 1000 python3 bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err; rc=$?
tail -3 gpurun_out/bench_final.err
exit $rc
