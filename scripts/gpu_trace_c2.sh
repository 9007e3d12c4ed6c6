#!/bin/bash
# Per-kernel times of the C2 invert (rocprofv3 kernel trace + stats) under the
# current defaults; output dir gpurun_out/$1.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-trace_c2}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
    python3 scripts/gpu_sweep.py SDP_HIP_DBG 0 > $out/run.log 2>&1 || exit $?
python3 - "$out" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:24]:
    print(f'{r["Name"][:90]:90s} calls {int(r["Calls"]):5d} avg {float(r["AverageNs"])/1e6:8.3f} ms')
PY
