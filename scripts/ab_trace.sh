#!/bin/bash
# rocprofv3 kernel stats of scripts/time_c2.py under library builds A/B
# (SDP_HIP_LIB_OVERRIDE; "" = the in-tree build); per-kernel averages printed.
#   scripts/ab_trace.sh tag [lib ...]      (extra time_c2.py args in TIME_ARGS)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tag=$1; shift
i=0
for L in "$@"; do
  i=$((i+1))
  out=gpurun_out/ab_${tag}_$i
  SDP_HIP_LIB_OVERRIDE=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
      python3 scripts/time_c2.py --reps 5 $TIME_ARGS > $out.log 2>&1 || { echo "run $i failed"; tail -5 $out.log; exit 1; }
  echo "== lib ${L:-in-tree}"
  python3 - "$out" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:24]:
        print(f"  {r['Name'].split('(')[0][:64]:64s} {int(r['Calls']):4d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
