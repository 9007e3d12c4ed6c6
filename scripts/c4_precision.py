"""C4 full band (13.4 Gvis, 8 streamed channel batches as bench.py's c4_n1)
accumulation-precision A/B: the dirty image against exact direct sums at
--npx pixels (tests/gpu_helpers.exact_pixels_dev, fp64 on the device) and
the adjointness <A x, y> = Re <x, A^H y> over every visibility, for each
library setting in --configs (env assignments, ';'-separated sets; '' =
defaults), each run --reps times.  One JSON line per run.

    python scripts/c4_precision.py --configs ";SDP_HIP_CORE=0;SDP_HIP_FOLD=0"
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gpu_helpers import exact_pixels_dev  # noqa: E402
from ska_sdp_func_python_amd import kernels, parallel, simulation  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default=";SDP_HIP_CORE=0;SDP_HIP_FOLD=0;SDP_HIP_CORE=0,SDP_HIP_FOLD=0")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--npx", type=int, default=64)
a = ap.parse_args()

dev = torch.device("cuda:0")
obs = simulation.device_observation(400, 1, 50e6, 350e6, config="LOW", device=dev,
                                    nchan_total=256, channels=[0])
uvw, nrow = obs["uvw"], obs["nrow"]
del obs["vis"], obs["wgt"]
freqs = np.linspace(50e6, 350e6, 256)
cell = 0.25 / obs["umax"]
npix = 8192
nb = max(-(-256 // 40), math.ceil(nrow * 256 / 1.8e9))
cuts = [256 * i // nb for i in range(nb + 1)]
batches = list(zip(cuts[:-1], cuts[1:]))
gen = torch.Generator(device=dev)
f_all = torch.as_tensor(freqs, device=dev)


def vis_of(lo, hi):
    gen.manual_seed(lo)
    return torch.randn((nrow, hi - lo), generator=gen, device=dev, dtype=torch.complex64)


rng = np.random.default_rng(90)
px = np.concatenate([[npix // 2, npix // 2 + 1], rng.integers(npix // 8, 7 * npix // 8, a.npx - 2)])
py = np.concatenate([[npix // 2 - 3, npix // 2], rng.integers(npix // 8, 7 * npix // 8, a.npx - 2)])
t0 = time.time()
flip = torch.tensor([-1.0, 1.0, -1.0], dtype=torch.float64, device=dev)
ex = np.zeros(a.npx)
for lo, hi in batches:
    ex += exact_pixels_dev(uvw * flip, freqs[lo:hi], vis_of(lo, hi), npix, cell, px, py)
print(json.dumps({"exact_pixels": a.npx, "s": round(time.time() - t0, 1)}), flush=True)

# the adjoint side once (the settings under test change only the gridder)
y = torch.zeros((npix, npix), dtype=torch.float64, device=dev)
iy = rng.integers(npix // 4, 3 * npix // 4, (2, 4096))
y[iy[0], iy[1]] = torch.as_tensor(rng.normal(size=4096), device=dev)
rhs = 0.0
for lo, hi in batches:
    v, _ = kernels.dirty2ms(uvw, f_all[lo:hi], y, None, cell, cell, 1e-7, True, flip_uw=True)
    x = vis_of(lo, hi)
    for r in range(0, nrow, 4_000_000):
        rhs += float(torch.sum((v[r:r + 4_000_000].to(torch.complex128).conj()
                                * x[r:r + 4_000_000].to(torch.complex128)).real))
    del v, x
torch.cuda.empty_cache()
kernels.release_workspace()

for cfg in a.configs.split(";"):
    env = dict(kv.split("=") for kv in cfg.split(",") if kv)
    for k, v in env.items():
        os.environ[k] = v
    for rep in range(a.reps):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        d = parallel.invert_batched_shard(uvw, f_all, vis_of, batches, npix, cell, 1e-7, True,
                                          flip_uw=True)  # RASCIL [y, x]
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t1) * 1e3
        dv = d.cpu().numpy()[py, px]
        e_px = float(np.sqrt(np.mean((dv - ex) ** 2) / np.mean(ex ** 2)))
        e_max = float(np.max(np.abs(dv - ex)) / np.sqrt(np.mean(ex ** 2)))
        lhs = float(torch.sum(d.T * y))
        print(json.dumps({"config": cfg or "default", "rep": rep, "ms_incl_vis_gen": round(ms, 1),
                          "px_rel_rms": e_px, "px_max_rel": e_max,
                          "adjointness": abs(lhs - rhs) / abs(lhs)}), flush=True)
        del d
    for k in env:
        os.environ.pop(k)
