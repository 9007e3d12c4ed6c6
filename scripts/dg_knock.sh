#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nufft_f64.py > gpurun_out/f64_tests.log 2>&1; rc=$?; tail -3 gpurun_out/f64_tests.log; exit $rc
