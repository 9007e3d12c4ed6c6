#!/bin/bash
# HBM traffic of one kernel per launch: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 --pmc passes (MI355X_MICROARCH.md HBM section), last dispatch of
# the kernels matching the regex, FETCH_SIZE doubled (gfx950 wide-read note).
#   scripts/pmc_traffic.sh <out.json> <kernel-regex> <command ...>
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
js=$1; rx=$2; shift 2
out=gpurun_out/traffic_$(basename "$js" .json)
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$rx" --output-format csv -d $out/$c -o run -- \
      "$@" > $out/$c.log 2>&1 || { echo "$c pass failed"; tail -5 $out/$c.log; exit 1; }
done
python3 - "$out" "$js" "$rx" <<'PY'
import csv, glob, json, os, sys
out, js, rx = sys.argv[1:4]
def last(sub, counter):
    vals, names = {}, {}
    for f in glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                d = int(r["Dispatch_Id"])
                vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
                names[d] = r["Kernel_Name"].split("(")[0]
    d = max(vals)
    return vals[d], names[d], len(vals)
fk, name, n = last("FETCH_SIZE", "FETCH_SIZE")
wk, _, _ = last("WRITE_SIZE", "WRITE_SIZE")
res = {"kernel": name, "regex": rx, "dispatches_seen": n, "fetch_size_kib": fk, "write_size_kib": wk,
       "bytes_per_launch": int(2 * fk * 1024 + wk * 1024),
       "note": "2 x FETCH_SIZE (gfx950 wide-read correction) + WRITE_SIZE, last dispatch"}
print(json.dumps(res))
json.dump(res, open(js, "w"), indent=1)
PY
