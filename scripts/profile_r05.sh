#!/bin/bash
# Round-5 evidence: rocprofv3 kernel stats + k_grid traffic of the default C2
# bench (profile.sh), the fp64 C2 kernel stats and traffic, the C2 degridder's
# traffic (the C4 gridding kernel is unchanged since r05_c4_kernel_stats.txt /
# traffic_c4_k_grid.json).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
set -o pipefail
bash scripts/profile.sh r05f > gpurun_out/prof_r05f.txt 2>&1 || { echo "profile.sh failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05f_f64 -o run -- \
    python3 scripts/time_c2.py --reps 3 --eps 1e-12 > gpurun_out/prof_r05f_f64.log 2>&1 || { echo "f64 trace failed"; exit 1; }
bash scripts/pmc_traffic.sh gpurun_out/traffic_k_grid_f64.json "k_grid_f64_mfma" \
    python3 scripts/time_c2.py --reps 1 --eps 1e-12 || exit 1
bash scripts/pmc_traffic.sh gpurun_out/traffic_k_degrid.json "k_degrid_mfma" \
    python3 scripts/time_c2.py --reps 1 || exit 1
echo done
