#!/bin/bash
# C4 N=1 (whole band on one GPU) and C2 stage timings: tree build vs variants
# (exp/*.so), and the tree with the plane zeroing serialised.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
run() {
  echo "== $1"
  timeout -k 10 200 python -u bench.py --config c4 --steps 2 --warmup 1 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print(json.dumps({'ms': d['ms_per_step'], 'Mvis_s': d['value'], 'stages': d['stages_ms_rank0']}))" || exit 1
  timeout -k 10 200 python scripts/gpu_sweep.py SDP_HIP_DUMMY 0,1 2>&1 | grep '^{' || exit 1
}
run tree || exit 1
SDP_HIP_ZERO_OVERLAP=0 run tree_zero_serial || exit 1
for v in "$@"; do SDP_HIP_LIB_OVERRIDE=$PWD/exp/$v.so run $v || exit 1; done
