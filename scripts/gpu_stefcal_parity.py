"""StefCal parity probe (GPU): measured gain / weight / residual deviation of
the device solve from (1) the reference-generated solve fixtures and (2) the
restated reference solver (oracle/ref_oracle.stefcal_row) on 512-station rows
drawn from the C5 distribution, with the iteration counts side by side."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ska-sdp-func-python_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ref_oracle as ro  # noqa: E402
from conftest import golden  # noqa: E402
from test_gpu_solvers import CASES, _tables  # noqa: E402
from ska_sdp_func_python_amd import kernels  # noqa: E402
from ska_sdp_func_python_amd.calibration import solve_gaintable  # noqa: E402

for case in CASES:
    g = golden(f"solve_{case}.npz")
    vis, model, gt = _tables(g)
    norm = str(g["normalise"])
    out = solve_gaintable(vis, model, gain_table=gt, phase_only=bool(g["phase_only"]),
                          niter=int(g["niter"]), tol=float(g["tol"]), crosspol=bool(g["crosspol"]),
                          normalise_gains=None if norm == "None" else norm, jones_type=str(g["jones"]))
    dg = np.max(np.abs(out["gain"].data - g["gain"]))
    dw = np.max(np.abs(out["weight"].data - g["weight"]) / np.maximum(np.abs(g["weight"]), 1e-30))
    dr = np.max(np.abs(out["residual"].data - g["residual"]))
    print(f"fixture {case:22s} max|dgain| {dg:.2e}  max rel dweight {dw:.2e}  max|dres| {dr:.2e}",
          flush=True)

nants, nchan = 512, 8
a1, a2 = np.triu_indices(nants, 1)
perm, conj, rs, ant2 = kernels.canonical_baselines(a1, a2, nants)
dev = torch.device("cuda:0")
rng = np.random.default_rng(1805550721)
for row in range(8):
    g = rng.lognormal(0, 0.1, (nants, nchan)) * np.exp(1j * rng.normal(0, 0.1, (nants, nchan)))
    xb = (g[a1] * np.conj(g[a2]))[..., None]
    xb = xb + 1e-3 * (rng.normal(size=xb.shape) + 1j * rng.normal(size=xb.shape))
    wb = rng.uniform(0.5, 1.5, xb.shape)
    gain = torch.ones((1, nants, nchan, 1, 1), dtype=torch.complex128, device=dev)
    gwt = torch.zeros((1, nants, nchan, 1, 1), dtype=torch.float64, device=dev)
    res, used = kernels.solve_gains(torch.as_tensor(xb[None, perm], device=dev),
                                    torch.as_tensor(wb[None, perm], device=dev), gain, gwt, rs,
                                    ant2, mode=0, niter=200, tol=1e-6, phase_only=False)
    t0 = time.time()
    eg, ew, er, eu = ro.stefcal_row(xb, wb, list(zip(a1, a2)), nants,
                                    np.ones((nants, nchan, 1, 1), complex),
                                    np.zeros((nants, nchan, 1, 1)), niter=200, tol=1e-6,
                                    phase_only=False)
    print(f"C5 row {row}: iterations gpu {int(used[0])} oracle {eu}; max|dgain| "
          f"{np.max(np.abs(gain[0].cpu().numpy() - eg)):.2e}; max rel dres "
          f"{np.max(np.abs(res[0].cpu().numpy() - er) / np.abs(er)):.2e} (oracle {time.time() - t0:.1f} s)",
          flush=True)
