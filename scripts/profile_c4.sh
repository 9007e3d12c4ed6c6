#!/bin/bash
# rocprofv3 kernel trace + stats of one C4 shard invert (scripts/bench_c4_shard.py)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_c4
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 scripts/bench_c4_shard.py --reps 1 "$@" > $out/c4_trace.log 2>&1 || exit $?
f=$(find $out/trace -name "run_kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:72]:72s} calls {int(r["Calls"]):5d}  avg {float(r["AverageNs"])/1e6:9.3f} ms  total {float(r["TotalDurationNs"])/1e6:9.2f} ms {100*float(r["TotalDurationNs"])/tot:5.1f}%')
PY
