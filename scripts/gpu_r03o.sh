#!/bin/bash
# r03o: rocprofv3 evidence for the current build (kernel stats + FETCH/WRITE
# passes), then the full GPU suite, smoke and the default bench line
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
bash scripts/profile.sh r03o || exit $?
bash scripts/gpu_session.sh r03o
