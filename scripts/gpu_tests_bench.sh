#!/bin/bash
# One GPU session: parity tests, smoke, short bench (each step time-limited).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
tag=${1:-run}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/${tag}_pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/${tag}_smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/${tag}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/${tag}_bench.log
exit $rc
