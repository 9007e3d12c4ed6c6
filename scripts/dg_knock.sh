#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
timeout -k 10 400 python3 bench.py --no-extra --steps 10 > gpurun_out/bench_cusplit.json 2> gpurun_out/bench_cusplit.err || { tail -20 gpurun_out/bench_cusplit.err; exit 1; }
