#!/bin/bash
# kernel trace of scripts/gpu_measure_paths.py for one path
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tag=${1:-trp}; shift
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
   python3 scripts/gpu_measure_paths.py "$@" > $out/log.txt 2>&1 || exit $?
python3 - "$out" <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-70s %5s %9.3f ms avg %9.3f tot" % (r["Name"][:70], r["Calls"], float(r["AverageNs"])/1e6, float(r["TotalDurationNs"])/1e6))
PY
