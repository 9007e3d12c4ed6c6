#!/bin/bash
# One GPU session: parity tests + smoke on the in-tree build, an A/B of the
# in-tree build against abvar/<variant>.so on the C2 step, the invert tests on
# the variant, then the default bench line.  Each GPU step has its own limit;
# the script stops at the first failure.
# usage: scripts/gpu_session.sh TAG [VARIANT] [PYTEST_K]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
tag=${1:-run}; var=${2:-}; kexpr=${3:-"ms2dirty or adjoint or linearity or batched or large_grid or fused or shared or c4_shard or c2_full_invert"}
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/${tag}_pytest.log; [ $rc -eq 0 ] || exit $rc
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_smoke.log
if [ -n "$var" ]; then
  step ab
  R=2 timeout -k 10 400 bash scripts/gpu_ab.sh cur abvar/$var.so > gpurun_out/${tag}_ab.txt 2>&1 || { cat gpurun_out/${tag}_ab.txt; exit 1; }
  cat gpurun_out/${tag}_ab.txt
  if [ "${VARTEST:-1}" = 1 ]; then
  step varpytest
  SDP_HIP_LIB_OVERRIDE=abvar/$var.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "$kexpr" > gpurun_out/${tag}_var_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${tag}_var_pytest.log; [ $rc -eq 0 ] || exit $rc
  fi
fi
if [ -n "$EXTRA" ]; then
  step extra
  timeout -k 10 900 bash $EXTRA || exit $?
fi
step bench
timeout -k 10 600 python bench.py > gpurun_out/${tag}_bench.log 2>&1
rc=$?; tail -c 3000 gpurun_out/${tag}_bench.log; step end; exit $rc
