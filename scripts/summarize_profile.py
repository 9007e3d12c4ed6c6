"""Summarise a scripts/profile.sh run: kernel stats table + k_grid HBM traffic.

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB.  Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE reports half the bytes of wide
coalesced reads on gfx950, so it is doubled; WRITE_SIZE counts float atomics
and 16-B stores exactly.  The gridding kernel's reads are 16-B + 8-B per lane
record loads (coalesced), so the x2 correction applies to them.
"""
import csv, glob, json, os, sys

out = sys.argv[1]


def rows(sub, name):
    f = glob.glob(os.path.join(out, sub, "**", name), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


print("== kernel stats (rocprofv3 --kernel-trace --stats, bench.py --steps 5 --warmup 2) ==")
for r in rows("trace", "run_kernel_stats.csv"):
    print("%-72s calls %4s  avg %9.3f ms  total %9.3f ms  %5.1f%%" % (
        r["Name"][:72], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6,
        float(r["Percentage"])))


def last_value(sub, counter):
    vals = {}
    for r in rows(sub, "run_counter_collection.csv"):
        if r["Counter_Name"] == counter and "k_grid" in r["Kernel_Name"]:
            d = int(r["Dispatch_Id"])
            vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return vals[max(vals)] if vals else None


fetch_kib = last_value("fetch", "FETCH_SIZE")
write_kib = last_value("write", "WRITE_SIZE")
res = {"kernel": "k_grid", "fetch_size_kib": fetch_kib, "write_size_kib": write_kib}
if fetch_kib is not None and write_kib is not None:
    res["bytes_per_launch"] = int(2 * fetch_kib * 1024 + write_kib * 1024)
    res["note"] = "2 x FETCH_SIZE (gfx950 wide-read correction) + WRITE_SIZE, last dispatch"
print("== k_grid HBM traffic per launch (PMC) ==")
print(json.dumps(res))
with open(os.path.join(out, "traffic_k_grid.json"), "w") as f:
    json.dump(res, f, indent=1)
