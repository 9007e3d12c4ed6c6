"""Summarise a scripts/gpu_c4_scaling.sh JSONL: per-N slowest emulated rank,
plus a modelled all-reduce of the 8192^2 fp64 image (537 MB; ring
all-reduce moves 2 (N-1)/N of it per GPU over xGMI at an assumed 150 GB/s
algorithm bandwidth per GPU for N = 8), against N = 1."""
import json
import sys

rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
n1 = [r for r in rows if "emulated_rank" not in r]
base = n1[0]["ms_per_step"] if n1 else None
IMG = 8192 * 8192 * 8
by = {}
for r in rows:
    if "emulated_rank" in r:
        # (the --c4-api lines before round 6's "partition" key: a rank holding
        # every channel is a rows-by-w rank)
        part = r.get("partition") or ("wrow" if r.get("block") == [0, 256] else "chan")
        if r.get("api"):
            part += "+api"
        by.setdefault((r["world"], part), []).append(r)
print(f"N=1: {base} ms")
for (w, part), rs in sorted(by.items()):
    mx = max(r["ms_per_step"] for r in rs)
    ar = 2 * (w - 1) / w * IMG / 150e9 * 1e3
    line = {"world": w, "partition": part, "ranks": len(rs),
            "rank_ms": [r["ms_per_step"] for r in sorted(rs, key=lambda r: r["emulated_rank"])],
            "model_ms": [r.get("model_ms") for r in sorted(rs, key=lambda r: r["emulated_rank"])],
            "max_rank_ms": mx, "allreduce_model_ms": round(ar, 2)}
    if base:
        line["speedup_no_allreduce"] = round(base / mx, 3)
        line["speedup_with_allreduce"] = round(base / (mx + ar), 3)
    print(json.dumps(line))
