#!/bin/bash
# NUFFT GPU tests, then C2 invert timings over the values of one env knob.
# usage: gpu_knob.sh tag KNOB v1,v2,... [notest]
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/$1; mkdir -p $out
if [ "$4" != notest ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_nufft.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 200 python scripts/gpu_sweep.py $2 $3 2>&1 | grep -v amdgpu.ids
