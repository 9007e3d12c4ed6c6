"""Dev probe: throughput of the non-metric paths at BASELINE.json sizes.

C2 predict (dirty2ms), C3 DFT (1000 comps x 10 Mvis), C5-shaped StefCal batch
(512 stations, B-type: per-channel solutions).  Prints one JSON line each.
"""
import json, math, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
import numpy as np, torch
from ska_sdp_func_python_amd import kernels, simulation

dev = torch.device("cuda:0")
which = sys.argv[1:] or ["predict", "dft", "stefcal"]


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), r


if "predict" in which:
    obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, device=dev)
    cell = 0.25 / obs["umax"]
    img = torch.randn(4096, 4096, dtype=torch.float64, device=dev)
    out = torch.empty_like(obs["vis"])
    kernels.set_stage_timing(True)
    t, (v, info) = timed(lambda: kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell,
                                                  1e-12, True, flip_uw=True, out=out))
    kernels.set_stage_timing(False)
    nvis = obs["nrow"] * 64
    print(json.dumps({"path": "predict C2 (dirty2ms)", "ms": round(t * 1e3, 3), "Mvis_s": round(nvis / t / 1e6, 1),
                      "stages": {k: round(info[k], 3) for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")},
                      "nitems": info["nitems"]}), flush=True)
    del obs, img, out, v

if "dft" in which:
    rng = np.random.default_rng(3)
    nbl, ntimes = 19306, 518
    fn_, n_def, lat, dec = simulation.CONFIGS["MID"]
    en = fn_(n_def, seed=1)
    ha = np.linspace(-0.5, 0.5, ntimes) * 8.0 * math.pi / 12.0
    uvw, _ = simulation.observe(en, math.radians(lat), math.radians(dec), ha)
    uvw = torch.as_tensor(uvw.reshape(-1, 3), device=dev)
    freq = torch.tensor([1.4e9], dtype=torch.float64, device=dev)
    ncomp = 1000
    lm = rng.uniform(-0.05, 0.05, (ncomp, 2))
    dc = torch.as_tensor(np.concatenate([lm, (np.sqrt(1 - (lm ** 2).sum(1)) - 1)[:, None]], 1), device=dev)
    flux = torch.as_tensor(rng.uniform(0.1, 10, (ncomp, 1, 1)).astype(complex), device=dev)
    out = torch.empty((uvw.shape[0], 1, 1), dtype=torch.complex64, device=dev)
    t, _ = timed(lambda: kernels.dft_point(dc, flux, uvw, freq=freq, out=out))
    nvis = uvw.shape[0]
    flops = nvis * ncomp * (6 + 8 * 1)
    print(json.dumps({"path": "DFT C3 (metres entry)", "nvis": nvis, "ncomp": ncomp, "ms": round(t * 1e3, 3),
                      "Mcompvis_s": round(nvis * ncomp / t / 1e6, 1), "TFLOP_s": round(flops / t / 1e12, 2)}), flush=True)
    uvwl = (uvw[:, None, :] * (freq / 299792458.0)[None, :, None]).contiguous()
    t2, _ = timed(lambda: kernels.dft_point(dc, flux, uvwl, out=out))
    print(json.dumps({"path": "DFT C3 (v00 uvw_lambda entry)", "ms": round(t2 * 1e3, 3),
                      "Mcompvis_s": round(nvis * ncomp / t2 / 1e6, 1)}), flush=True)
    del uvw, uvwl, out

if "stefcal" in which:
    nants, nchan = 512, 64
    ntime = int(os.environ.get("STEFCAL_NTIME", "8"))
    a1, a2 = np.triu_indices(nants, 1)
    rng = np.random.default_rng(1805550721)
    g = (rng.lognormal(0, 0.1, (ntime, nants, nchan)) * np.exp(1j * rng.normal(0, 0.1, (ntime, nants, nchan))))
    perm, conj, rs, ant2 = kernels.canonical_baselines(a1, a2, nants)
    gt = torch.as_tensor(g, device=dev)
    a1t = torch.as_tensor(a1[perm], device=dev); a2t = torch.as_tensor(a2[perm], device=dev)
    xb = (gt[:, a1t, :] * torch.conj(gt[:, a2t, :]))[..., None].contiguous()   # [t, nbl, nchan, 1]
    wb = torch.ones(xb.shape, dtype=torch.float64, device=dev)
    def run():
        gain = torch.ones((ntime, nants, nchan, 1, 1), dtype=torch.complex128, device=dev)
        gwt = torch.zeros((ntime, nants, nchan, 1, 1), dtype=torch.float64, device=dev)
        return kernels.solve_gains(xb, wb, gain, gwt, rs, ant2, mode=0, niter=200, tol=1e-6, phase_only=False)
    t, (res, used) = timed(run)
    nsub = ntime * nchan
    iters = int(used.max())
    nbl = len(a1)
    print(json.dumps({"path": f"StefCal C5-shaped batch (B jones: per-chan solutions, {ntime} times x {nchan} chans)",
                      "nants": nants, "nbl": nbl, "sub_solves": nsub, "iterations": iters, "ms": round(t * 1e3, 3),
                      "solves_s": round(nsub / t, 1), "iter_GBs": round(12 * nbl * nsub * iters / t / 1e9, 1),
                      "max_residual": float(res.max())}), flush=True)
