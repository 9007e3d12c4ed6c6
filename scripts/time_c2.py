"""C2 invert and predict wall times (median of --reps after a warm-up), for
A/B of library variants: python scripts/time_c2.py [--reps N] [--eps E]."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ska_sdp_func_python_amd import kernels, simulation  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=7)
ap.add_argument("--eps", type=float, default=1e-7, help="1e-7: fp32 NUFFT; 1e-12: fp64")
a = ap.parse_args()
dev = torch.device("cuda:0")
obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, config="MID", seed=0, device=dev)
cell = 0.25 / obs["umax"]
img = torch.randn(4096, 4096, dtype=torch.float64, device=dev)
res = {}
for name in ("invert", "predict"):
    kernels.set_stage_timing(True)
    ts, infos = [], []
    for i in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if name == "invert":
            _, info = kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], 4096, 4096,
                                       cell, cell, a.eps, True, flip_uw=True)
        else:
            _, info = kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell, a.eps,
                                       True, flip_uw=True)
        torch.cuda.synchronize()
        if i:
            ts.append(time.perf_counter() - t0)
            infos.append(info)
    kernels.set_stage_timing(False)
    res[name] = {"ms": round(1e3 * float(np.median(ts)), 3),
                 **{k: round(float(np.median([x[k] for x in infos])), 3)
                    for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")},
                 **{k: infos[-1][k] for k in ("support", "nplanes", "nitems", "nvis_used")}}
print(json.dumps(res))
