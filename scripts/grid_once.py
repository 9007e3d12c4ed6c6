"""One C2 invert (bench.py's workload: 123.6 Mvis, 4096^2 image, 8192^2 grid)
repeated --reps times: the driver for rocprofv3 PMC passes on the gridder."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))

import torch  # noqa: E402

from ska_sdp_func_python_amd import kernels, simulation  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--predict", action="store_true")
ap.add_argument("--c4", action="store_true",
                help="C4 top channel block (32 of 256 channels, 1.67 Gvis, 8192^2 image)")
a = ap.parse_args()
dev = torch.device("cuda:0")
npix = 4096
if a.c4:
    npix = 8192
    obs = simulation.device_observation(400, 32, 50e6, 350e6, config="LOW", device=dev,
                                        nchan_total=256, channels=list(range(224, 256)))
else:
    obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, config="MID", seed=0, device=dev)
cell = 0.25 / obs["umax"]
img = torch.randn(npix, npix, dtype=torch.float64, device=dev)
for _ in range(a.reps):
    if a.predict:
        kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell, 1e-7, True,
                         flip_uw=True)
    else:
        kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], npix, npix, cell, cell,
                         1e-7, True, flip_uw=True)
torch.cuda.synchronize()
print("done")
