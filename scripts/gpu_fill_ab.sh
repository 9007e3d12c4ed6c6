#!/bin/bash
# k_fill tile A/B: solver parity on the variant, then C5-slice kernel stats (tree = 64-wide tiles vs exp/v_fill32.so).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_fullsize.py::test_c5_full_batch_and_sampled_rows -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/fill64_pytest.log 2>&1 || { tail -30 gpurun_out/fill64_pytest.log; exit 1; }
tail -1 gpurun_out/fill64_pytest.log
for v in tree v_fill32 tree v_fill32; do
  if [ $v = tree ]; then unset SDP_HIP_LIB_OVERRIDE; else export SDP_HIP_LIB_OVERRIDE=$PWD/exp/$v.so; fi
  rm -rf gpurun_out/prof_fill
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fill -o c5 -- python3 bench.py --config c5 --c5-times 96 --steps 1 --warmup 1 > gpurun_out/prof_fill.log 2>&1 || exit $?
  python3 -c "import csv; [print('== $v', r['Name'][:22], r['Calls'], float(r['AverageNs']) / 1e6) for r in csv.DictReader(open('gpurun_out/prof_fill/c5_kernel_stats.csv')) if 'k_fill' in r['Name'] or 'k_iter' in r['Name']]"
done
