#!/bin/bash
# r03m: the gridder flush without branches (per-plane descriptors hoisted,
# out-of-range planes and zero floats dropped by the buffer range check):
# C2 invert A/B (in-tree HEAD build vs abvar/gflush.so), C4 N=1 A/B, then the
# NUFFT parity tests on gflush
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
R=2 bash scripts/gpu_ab.sh cur abvar/gflush.so || exit 1
c4() {
  timeout -k 10 300 python -u bench.py --config c4 --steps 1 --warmup 1 --c4-cpu-chans 0 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$1', json.dumps({'ms': d['ms_per_step'], 'Mvis_s': d['value'], 'stages': d.get('stages_ms_rank0')}))"
}
c4 cur || exit 1
SDP_HIP_LIB_OVERRIDE=abvar/gflush.so c4 gflush || exit 1
SDP_HIP_LIB_OVERRIDE=abvar/gflush.so timeout -k 10 600 python -u -m pytest tests/test_gpu_nufft.py tests/test_gpu_fullsize.py tests/test_gpu_orientation.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03m_pytest.log 2>&1 || { tail -30 gpurun_out/r03m_pytest.log; exit 1; }
tail -1 gpurun_out/r03m_pytest.log
