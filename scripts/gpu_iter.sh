#!/bin/bash
# quick iteration: NUFFT GPU tests + knob sweep
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
tag=${1:-iter}; shift
timeout -k 10 600 python -m pytest tests/test_gpu_nufft.py -q -x -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/${tag}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python scripts/gpu_sweep.py "$@" > gpurun_out/${tag}_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/${tag}_sweep.log | grep -v amdgpu.ids
exit $rc
