"""Dev probe: one C5-shaped StefCal batch (512 stations, 64 x 64 sub-solves,
20 iterations) for PMC passes on k_iter."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
import numpy as np, torch
from ska_sdp_func_python_amd import kernels

dev = torch.device("cuda:0")
nants, nchan, ntime = 512, 64, 64
a1, a2 = np.triu_indices(nants, 1)
rng = np.random.default_rng(1805550721)
g = rng.lognormal(0, 0.1, (ntime, nants, nchan)) * np.exp(1j * rng.normal(0, 0.1, (ntime, nants, nchan)))
perm, conj, rs, ant2 = kernels.canonical_baselines(a1, a2, nants)
gt = torch.as_tensor(g, device=dev)
a1t, a2t = torch.as_tensor(a1[perm], device=dev), torch.as_tensor(a2[perm], device=dev)
xb = (gt[:, a1t, :] * torch.conj(gt[:, a2t, :]))[..., None].contiguous()
wb = torch.ones(xb.shape, dtype=torch.float64, device=dev)
for rep in range(2):
    gain = torch.ones((ntime, nants, nchan, 1, 1), dtype=torch.complex128, device=dev)
    gwt = torch.zeros((ntime, nants, nchan, 1, 1), dtype=torch.float64, device=dev)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    res, used = kernels.solve_gains(xb, wb, gain, gwt, rs, ant2, mode=0, niter=200, tol=1e-6,
                                    phase_only=False)
    torch.cuda.synchronize()
    print(f"rep {rep}: {(time.perf_counter() - t0) * 1e3:.2f} ms, iters {int(used.max())}", flush=True)
