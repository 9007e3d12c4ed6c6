"""C3's sky-component DFT (1000 point components x 10 Mvis, stokesI, c64
output, one channel as bench.py --config c3) run --reps times: the driver
for rocprofv3 PMC passes on k_dft_mfma."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))

import torch  # noqa: E402

from ska_sdp_func_python_amd import kernels  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--ncomp", type=int, default=1000)
ap.add_argument("--nvis", type=int, default=10_000_000)
ap.add_argument("--nchan", type=int, default=1)
ap.add_argument("--c128", action="store_true", help="complex128 output (the fp64 path)")
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
g.manual_seed(3)
nchan = a.nchan
nrow = a.nvis // nchan
uvw = (torch.rand((nrow, 3), dtype=torch.float64, device=dev, generator=g) - 0.5) * 2e4
uvw[:, 2] *= 0.2
freq = torch.linspace(1.0e9, 1.2e9, nchan, dtype=torch.float64, device=dev)
lmn = (torch.rand((a.ncomp, 3), dtype=torch.float64, device=dev, generator=g) - 0.5) * 0.05
lmn[:, 2] = torch.sqrt(1 - lmn[:, 0] ** 2 - lmn[:, 1] ** 2) - 1
flux = torch.rand((a.ncomp, 1, 1), dtype=torch.float64, device=dev, generator=g).to(torch.complex128)
out = torch.empty((nrow, nchan, 1), dtype=torch.complex128 if a.c128 else torch.complex64,
                  device=dev)
import time  # noqa: E402
for _ in range(a.reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernels.dft_point(lmn, flux, uvw, freq, out)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{'c128' if a.c128 else 'c64'} {1e3 * dt:.3f} ms = "
          f"{a.ncomp * nrow * nchan / dt / 1e9:.1f} G comp*vis/s", flush=True)
print("done", float(out.abs().sum()))
