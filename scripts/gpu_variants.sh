#!/bin/bash
# A/B of kernel variants built by scripts/build_variants.sh: NUFFT parity tests
# on the first variant, then C2 invert timings for every variant (+ the
# in-tree build with SDP_HIP_GRID_V1, the previous gridder).
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/${1:-var}; shift
mkdir -p $out
lib_for() { [ "$1" = tree ] || echo "$PWD/exp/$1.so"; }  # "tree": the in-tree build
first=$1
if [ "$first" = notest ]; then shift; else
SDP_HIP_LIB_OVERRIDE=$(lib_for $first) timeout -k 10 400 python -u -m pytest tests/test_gpu_nufft.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1
rc=$?; echo "pytest($first) rc=$rc"; tail -3 $out/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
SDP_HIP_GRID_V1=1 timeout -k 10 120 python scripts/gpu_sweep.py SDP_HIP_DBG ${VALS:-0} 2>&1 | grep -v amdgpu.ids | sed 's/^/V1 /' || exit 1
for v in "$@"; do
  SDP_HIP_LIB_OVERRIDE=$(lib_for $v) timeout -k 10 120 python scripts/gpu_sweep.py SDP_HIP_DBG ${VALS:-0} 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit 1
done
