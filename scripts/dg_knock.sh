#!/bin/bash
# GPU suite + C2 timings on the current build
cd "$(dirname "$0")/.." || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=5 > gpurun_out/gpu_suite.log 2>&1; rc=$?
tail -12 gpurun_out/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/time_c2.py --reps 7 || exit 1
timeout -k 10 200 python3 scripts/time_c2.py --reps 3 --eps 1e-12 || exit 1
