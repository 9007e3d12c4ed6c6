#!/bin/bash
# Invert parity tests on the tree build, then a C2 stage sweep over one env knob.
# usage: scripts/gpu_knob_ab.sh KNOB v1,v2[,...] [pytest -k expression]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
knob=$1; vals=$2; kexp=${3:-"ms2dirty or invert or adjoint or linearity or chunking or batched"}
timeout -k 10 400 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_fullsize.py::test_c2_full_invert_against_reference_precision -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$kexp" > gpurun_out/knob_pytest.log 2>&1 || { tail -30 gpurun_out/knob_pytest.log; exit 1; }
tail -1 gpurun_out/knob_pytest.log
timeout -k 10 300 python scripts/gpu_sweep.py $knob $vals 2>&1 | grep -v amdgpu.ids
