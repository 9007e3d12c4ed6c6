#!/bin/bash
# C4 / predict parity on the tree build, then A/B of variants (exp/*.so) on a
# C4 rank block (rank 7 of 8) and the C2 predict path; C4 N=1 line last.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_fullsize.py::test_c4_shard_invert_predict_at_full_size -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "large_grid or subsort or predict or dirty2ms or c4 or round_trip" > gpurun_out/c4ab_pytest.log 2>&1 || { tail -30 gpurun_out/c4ab_pytest.log; exit 1; }
tail -1 gpurun_out/c4ab_pytest.log
for v in tree "$@"; do
  if [ $v = tree ]; then unset SDP_HIP_LIB_OVERRIDE; else export SDP_HIP_LIB_OVERRIDE=$PWD/exp/$v.so; fi
  echo "== $v"
  timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --emulate 7/8 2>&1 | grep '^{' || exit 1
  timeout -k 10 300 python scripts/bench_paths.py predict 2>&1 | grep '^{' | cut -c1-260 || exit 1
done
unset SDP_HIP_LIB_OVERRIDE
timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 > gpurun_out/c4_n1.log 2>&1 || exit $?
grep '^{' gpurun_out/c4_n1.log
