#!/bin/bash
# r03g: the row-partition GPU test, then C4 N = 1 and the 8 ranks of the 8-way
# row-by-w partition emulated one at a time
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_nufft.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "row_partition" > gpurun_out/r03g_pytest.log 2>&1 || { tail -30 gpurun_out/r03g_pytest.log; exit 1; }
tail -1 gpurun_out/r03g_pytest.log
WORLDS=${WORLDS:-8} C4ARGS="--partition wrow" bash scripts/gpu_c4_scaling.sh r03g > gpurun_out/r03g_c4.log 2>&1 || { tail -30 gpurun_out/r03g_c4.log; exit 1; }
python3 scripts/c4_scaling_summary.py gpurun_out/r03g_c4_scaling.jsonl
