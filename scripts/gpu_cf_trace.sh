#!/bin/bash
# rocprofv3 kernel stats of the CF (AW-projection) gridding bench case.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-prof_cf}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
    python3 scripts/bench_paths.py cfgrid > $out/run.log 2>&1 || exit $?
python3 - "$out" <<'PY' > $out/summary.txt
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
print("== kernel stats: rocprofv3 --kernel-trace --stats -- bench_paths.py cfgrid (4 Mvis x 64 taps, 4096^2) ==")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:70]:70s} calls {int(r["Calls"]):5d} avg {float(r["AverageNs"])/1e6:8.3f} ms')
PY
cat $out/summary.txt
