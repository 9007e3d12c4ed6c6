#!/bin/bash
# r03e: C2 rocprof kernel stats + HBM traffic (profile.sh), gridder PMC
# counters (pmc_grid.sh), then the C4 channel-block 8-way emulation
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
echo "== profile $(date +%T)"
bash scripts/profile.sh r03e > gpurun_out/r03e_profile.log 2>&1 || { tail -30 gpurun_out/r03e_profile.log; exit 1; }
tail -40 gpurun_out/r03e_profile.log
echo "== pmc $(date +%T)"
bash scripts/pmc_grid.sh r03e_pmc k_grid > gpurun_out/r03e_pmc.log 2>&1 || { tail -30 gpurun_out/r03e_pmc.log; exit 1; }
tail -25 gpurun_out/r03e_pmc.log
echo "== c4 chan 8-way $(date +%T)"
WORLDS=8 C4ARGS="--partition chan" bash scripts/gpu_c4_scaling.sh r03e > gpurun_out/r03e_c4.log 2>&1 || { tail -30 gpurun_out/r03e_c4.log; exit 1; }
python3 scripts/c4_scaling_summary.py gpurun_out/r03e_c4_scaling.jsonl
echo "== end $(date +%T)"
