#!/bin/bash
# the -m gpu suite on the current build -> gpurun_out/gpu_suite.log
cd "$(dirname "$0")/.." || exit 1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=5 > gpurun_out/gpu_suite.log 2>&1; rc=$?
tail -12 gpurun_out/gpu_suite.log
exit $rc
