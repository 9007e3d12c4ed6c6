"""Dev probe: C2 invert stage timings under different kernel knobs (env vars)."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
import numpy as np, torch
from ska_sdp_func_python_amd import kernels, simulation

dev = torch.device("cuda:0")
nchan = int(os.environ.get("SWEEP_NCHAN", "64"))
obs = simulation.device_observation(100, nchan, 0.95e9, 1.76e9, device=dev, nchan_total=64,
                                    channels=np.arange(nchan) if nchan < 64 else None)
cell = 0.25 / obs["umax"]
if os.environ.get("SWEEP_BLMAJOR") == "1":
    # rows [time][baseline] -> [baseline][time] (experiment: traversal order)
    nbl = 197 * 196 // 2
    nt = obs["nrow"] // nbl
    perm = torch.arange(obs["nrow"], device=dev).reshape(nt, nbl).t().reshape(-1)
    for k in ("uvw", "vis", "wgt"):
        obs[k] = obs[k][perm].contiguous()
npix = 4096
knob = sys.argv[1] if len(sys.argv) > 1 else "SDP_HIP_GRID_WAVES"
vals = sys.argv[2].split(",") if len(sys.argv) > 2 else ["1", "2", "4"]
kernels.set_stage_timing(True)
ref = None
for v in vals:
    os.environ[knob] = v
    res = []
    for it in range(4):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        img, info = kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], npix, npix,
                                     cell, cell, 1e-12, True, flip_uw=True)
        torch.cuda.synchronize(); t1 = time.perf_counter()
        if it > 0:
            res.append(((t1 - t0) * 1e3, info["ms_prep"], info["ms_grid"], info["ms_fft"], info["ms_screen"]))
    a = img.cpu().numpy()
    if ref is None:
        ref = a
    err = float(np.sqrt(np.mean((a - ref) ** 2) / np.mean(ref ** 2)))
    m = np.mean(res, axis=0)
    print(json.dumps({knob: v, "wall_ms": round(m[0], 3), "prep": round(m[1], 3), "grid": round(m[2], 3),
                      "fft": round(m[3], 3), "screen": round(m[4], 3), "nitems": info["nitems"],
                      "rel_vs_first": err, "Mvis_s": round(obs["nrow"] * nchan / m[0] / 1e3, 1)}), flush=True)
