"""C2 4-pol predict at the kernel API, alternated in one process: one
dirty2ms_vis call per image pol (stokesIQUV -> linear columns, accumulating
after the first) against one dirty2ms_vis_pols call; c128 output
[nrow, nchan, 4].  Prints each timing and the relative RMS difference."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))

import torch  # noqa: E402

from ska_sdp_func_python_amd import kernels, simulation  # noqa: E402

dev = torch.device("cuda:0")
obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, config="MID", seed=0, device=dev)
cell = 0.25 / obs["umax"]
nrow, nchan = obs["uvw"].shape[0], obs["vis"].shape[1]
imgs = torch.randn(4, 4096, 4096, dtype=torch.float64, device=dev)
cols = [[1, 0, 0, 1], [1, 0, 0, -1], [0, 1, 1, 0], [0, 1j, -1j, 0]]
a = torch.empty((nrow, nchan, 4), dtype=torch.complex128, device=dev)
b = torch.empty_like(a)


def per_pol():
    for q in range(4):
        kernels.dirty2ms_vis(obs["uvw"], obs["freq"], imgs[q], a, cols[q], cell, cell, 1e-7, True,
                             flip_uw=True, accumulate=q > 0)


def pols():
    kernels.dirty2ms_vis_pols(obs["uvw"], obs["freq"], imgs, b, cols, cell, cell, 1e-7, True,
                              flip_uw=True)


for f in (per_pol, pols):
    f()
for r in range(3):
    for name, f in (("per_pol", per_pol), ("pols", pols)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        print(f"{name} {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
d = (a - b).abs().pow(2).mean().sqrt() / a.abs().pow(2).mean().sqrt()
print(f"rel rms difference {float(d):.3e}")
