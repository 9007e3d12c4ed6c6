"""invert_ng through the reference-shaped API on a device-resident C2
Visibility (vis c128, imaging_weight f64, flags int64: the datamodels'
dtypes), against the bare C-ABI call that bench.py times.  The difference is
the vis-side prologue (flag masking, dtype conversion, pol conversion,
sumwt) -- SURVEY.md §8(f) rank 2.

usage: python scripts/bench_invert_api.py [npol(1|4)] [nchan]
"""
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ska_sdp_func_python_amd import datamodels as dm, kernels, simulation  # noqa: E402
from ska_sdp_func_python_amd.imaging import invert_ng, predict_ng  # noqa: E402

npol = int(sys.argv[1]) if len(sys.argv) > 1 else 1
nchan = int(sys.argv[2]) if len(sys.argv) > 2 else 64
dev = torch.device("cuda:0")
obs = simulation.device_observation(100, nchan, 0.95e9, 1.76e9, device=dev)
nrow = obs["nrow"]
nb = 197 * 196 // 2
nt = nrow // nb
cell = 0.25 / obs["umax"]
pf = dm.PolarisationFrame("stokesI" if npol == 1 else "linear")
ipf = dm.PolarisationFrame("stokesI" if npol == 1 else "stokesIQUV")
g = torch.Generator(device=dev)
g.manual_seed(2)
vis = torch.randn((nt, nb, nchan, npol), dtype=torch.complex128, device=dev, generator=g)
shape = vis.shape
pc = dm.SkyCoord(0.0, math.radians(-30.0))
bvis = dm.Visibility.constructor(
    frequency=obs["freq"].cpu().numpy(), channel_bandwidth=np.full(nchan, 1e6), phasecentre=pc,
    uvw=obs["uvw"].reshape(nt, nb, 3), time=np.arange(nt, dtype=float),
    vis=vis, weight=torch.ones(shape, dtype=torch.float64, device=dev),
    imaging_weight=torch.ones(shape, dtype=torch.float64, device=dev),
    flags=torch.zeros(shape, dtype=torch.int64, device=dev),
    baselines=np.stack(np.triu_indices(197, 1), 1), polarisation_frame=pf)
del obs
f = np.asarray(bvis.frequency.data)
model = dm.create_image(4096, cell, pc, polarisation_frame=ipf, frequency=float(f.mean()),
                        channel_bandwidth=float(2 * (f.max() - f.min()) + 1e6), nchan=1)


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


t_api = timed(lambda: invert_ng(bvis, model, epsilon=1e-12))
uvw = bvis.uvw.data.reshape(-1, 3).contiguous()
freq = torch.as_tensor(f, device=dev)
ms = bvis.vis.data.reshape(nrow, nchan, npol)[:, :, 0].to(torch.complex64).contiguous()
wgt = torch.ones((nrow, nchan), dtype=torch.float32, device=dev)
out = torch.zeros((4096, 4096), dtype=torch.float64, device=dev)
t_kernel = timed(lambda: kernels.ms2dirty(uvw, freq, ms, wgt, 4096, 4096, cell, cell, 1e-12, True,
                                          flip_uw=True, out=out, out_strides=(1, 4096)))
model["pixels"].data = torch.randn((1, npol, 4096, 4096), dtype=torch.float64, device=dev)
t_pred = timed(lambda: predict_ng(bvis, model, epsilon=1e-12))
img = model["pixels"].data[0, 0]
vout = torch.empty((nrow, nchan), dtype=torch.complex64, device=dev)
t_dk = timed(lambda: kernels.dirty2ms(uvw, freq, img, None, cell, cell, 1e-12, True, flip_uw=True,
                                      out=vout, dirty_strides=(1, 4096), npix=(4096, 4096)))
print(json.dumps({"npol": npol, "nchan": nchan, "nvis": nrow * nchan,
                  "invert_ng_ms": round(t_api * 1e3, 2),
                  "ms2dirty_per_pol_ms": round(t_kernel * 1e3, 2),
                  "prologue_overhead_ms": round((t_api - npol * t_kernel) * 1e3, 2),
                  "predict_ng_ms": round(t_pred * 1e3, 2),
                  "dirty2ms_per_pol_ms": round(t_dk * 1e3, 2),
                  "predict_overhead_ms": round((t_pred - npol * t_dk) * 1e3, 2)}))
