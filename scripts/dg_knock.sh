#!/bin/bash
# 4-pol invert_ng at eps 1e-12: HEAD lib (kept single-level bucketing, VALU fp64 gridder) vs in-tree
cd "$(dirname "$0")/.." || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nufft.py -k "fused_prologue" > gpurun_out/pol_tests.log 2>&1; rc=$?; tail -2 gpurun_out/pol_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== in-tree"; timeout -k 10 300 python3 scripts/pol4_f64.py || exit 1
echo "== HEAD lib + keep (the old invert_ng)"; SDP_HIP_LIB_OVERRIDE=abtmp/lib_head.so timeout -k 10 300 python3 -c "
import sys; sys.argv=['x']; sys.path.insert(0, 'ska-sdp-func-python_amd')
from ska_sdp_func_python_amd import kernels
kernels.is_fp64 = lambda *a, **k: False
exec(open('scripts/pol4_f64.py').read())" || exit 1
