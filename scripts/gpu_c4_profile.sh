#!/bin/bash
# rocprofv3 kernel stats of one C4 rank (the 8-way partition's last block,
# the most w planes) through bench.py --config c4 --emulate.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-prof_c4}
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
    python3 bench.py --config c4 --emulate 7/8 --steps 1 --warmup 1 > $out/bench.log 2>&1 || exit $?
python3 - "$out" <<'PY' > $out/summary.txt
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("== kernel stats: rocprofv3 --kernel-trace --stats -- bench.py --config c4 --emulate 7/8 --steps 1 --warmup 1 ==")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:24]:
    print(f'{r["Name"][:72]:72s} calls {int(r["Calls"]):5d} avg {float(r["AverageNs"])/1e6:9.3f} ms total {float(r["TotalDurationNs"])/1e6:9.1f} ms {100*float(r["TotalDurationNs"])/tot:5.1f}%')
PY
cat $out/summary.txt
