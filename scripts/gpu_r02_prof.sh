#!/bin/bash
# predict parity + path line, C2 profile (trace + PMC traffic), C3 kernel stats.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_fullsize.py::test_c2_full_predict_against_reference_precision -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "dirty2ms or predict or adjoint or round_trip" > gpurun_out/pf_pytest.log 2>&1 || { tail -30 gpurun_out/pf_pytest.log; exit 1; }
tail -1 gpurun_out/pf_pytest.log
timeout -k 10 300 python scripts/bench_paths.py predict > gpurun_out/predict_path2.log 2>&1 || exit $?
tail -1 gpurun_out/predict_path2.log
bash scripts/profile.sh r02b || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --config c3 --steps 10 --warmup 2 > gpurun_out/c3_prof_bench.log 2>&1 || exit $?
find gpurun_out/prof_c3 -name "*stats*"
