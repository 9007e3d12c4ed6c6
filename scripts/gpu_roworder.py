"""Dev probe: invert time with time-major vs baseline-major row order (same data)."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
import numpy as np, torch
from ska_sdp_func_python_amd import kernels, simulation
dev = torch.device("cuda:0")
obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, device=dev)
cell = 0.25 / obs["umax"]
nt, nb = 100, obs["nrow"] // 100
bl = {k: obs[k].view(nt, nb, -1).transpose(0, 1).reshape(nt * nb, -1).contiguous() for k in ("uvw", "vis", "wgt")}
kernels.set_stage_timing(True)
for name, d in (("time-major", obs), ("baseline-major", bl)):
    for it in range(4):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        img, info = kernels.ms2dirty(d["uvw"], obs["freq"], d["vis"], d["wgt"], 4096, 4096, cell, cell, 1e-12, True, flip_uw=True)
        torch.cuda.synchronize(); t = time.perf_counter() - t0
    print(json.dumps({"order": name, "wall_ms": round(t * 1e3, 3), **{k: round(info[k], 3) for k in ("ms_prep", "ms_grid", "ms_fft")}}))
