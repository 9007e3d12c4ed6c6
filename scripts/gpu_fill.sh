#!/bin/bash
# StefCal parity after the k_fill change, C5 line, k_fill kernel statistics.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_fullsize.py::test_c5_full_batch_and_sampled_rows tests/test_gpu_skymodel.py tests/test_gpu_parallel.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/fill_pytest.log 2>&1 || { tail -30 gpurun_out/fill_pytest.log; exit 1; }
tail -1 gpurun_out/fill_pytest.log
timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 0 > gpurun_out/fill_c5.log 2>&1 || exit $?
grep '^{' gpurun_out/fill_c5.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5b -o c5 -- python3 bench.py --config c5 --c5-times 96 --steps 1 --warmup 1 > gpurun_out/prof_c5b.log 2>&1 || exit $?
grep -E "k_fill|k_iter|k_residual" gpurun_out/prof_c5b/c5_kernel_stats.csv | cut -c1-40,150-260
