#!/bin/bash
# r03r: polynomial ES taps in the padded gridder (in-tree build) -- the full
# GPU suite and smoke on it, C2 invert A/B against abvar/nopoly.so (the same
# source built with -DSDP_ES_POLY=0), C4 N=1 A/B, then the default bench line.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03r_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03r_pytest.log; [ $rc -eq 0 ] || exit $rc
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03r_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r03r_smoke.log
step ab_c2
R=3 timeout -k 10 500 bash scripts/gpu_ab.sh cur abvar/nopoly.so > gpurun_out/r03r_ab_c2.txt 2>&1 || { cat gpurun_out/r03r_ab_c2.txt; exit 1; }
cat gpurun_out/r03r_ab_c2.txt
step ab_c4
for v in cur abvar/nopoly.so cur; do
  if [ $v = cur ]; then L=""; else L="SDP_HIP_LIB_OVERRIDE=$PWD/$v"; fi
  env $L timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --c4-cpu-chans 0 > gpurun_out/r03r_c4_ab.log 2>&1 || { tail -20 gpurun_out/r03r_c4_ab.log; exit 1; }
  grep '^{' gpurun_out/r03r_c4_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['stages_ms_rank0'])" | tee -a gpurun_out/r03r_ab_c4.txt
done
step bench
timeout -k 10 600 python bench.py > gpurun_out/r03r_bench.log 2>&1
rc=$?; tail -c 1500 gpurun_out/r03r_bench.log; step end; exit $rc
