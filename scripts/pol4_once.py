"""The bench's 4-pol MFS invert_ng (linear c128 / f64 / int64 Visibility of
the C2 layout -> stokesIQUV, eps 1e-7) run --reps times, or with --predict
predict_ng of a random stokesIQUV model into that Visibility: the driver for
timings and rocprofv3 kernel traces of the multi-pol paths."""
import argparse
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))

import torch  # noqa: E402

from ska_sdp_func_python_amd import datamodels as dm, simulation  # noqa: E402
from ska_sdp_func_python_amd.imaging import invert_ng, predict_ng  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--predict", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, config="MID", seed=0, device=dev)
cell = 0.25 / obs["umax"]
nrow, nchan = obs["uvw"].shape[0], obs["vis"].shape[1]
nb = 197 * 196 // 2
nt = nrow // nb
s4 = (nt, nb, nchan, 4)
pc = dm.SkyCoord(0.0, math.radians(-45.0))
freq = obs["freq"].cpu().numpy()
v4 = obs["vis"].to(torch.complex128).reshape(nt, nb, nchan, 1).expand(s4).contiguous()
w4 = torch.ones(s4, dtype=torch.float64, device=dev)
b4 = dm.Visibility.constructor(
    frequency=freq, channel_bandwidth=np.full(nchan, 1e6), phasecentre=pc,
    uvw=obs["uvw"].reshape(nt, nb, 3), time=np.arange(nt, dtype=float), vis=v4, weight=w4,
    imaging_weight=w4, flags=torch.zeros(s4, dtype=torch.int64, device=dev),
    baselines=np.stack(np.triu_indices(197, 1), 1), polarisation_frame=dm.PolarisationFrame("linear"))
m4 = dm.create_image(4096, cell, pc, polarisation_frame=dm.PolarisationFrame("stokesIQUV"),
                     frequency=float(freq.mean()),
                     channel_bandwidth=float(2 * (freq.max() - freq.min()) + 1e6), nchan=1)
if a.predict:
    m4["pixels"].data = torch.randn(1, 4, 4096, 4096, dtype=torch.float64, device=dev)
for i in range(a.reps):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if a.predict:
        predict_ng(b4, m4, epsilon=1e-7)
    else:
        invert_ng(b4, m4, epsilon=1e-7)
    torch.cuda.synchronize(dev)
    print(f"4-pol {'predict_ng' if a.predict else 'invert_ng'} "
          f"{1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
