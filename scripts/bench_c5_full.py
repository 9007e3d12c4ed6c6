"""C5 measured end to end on one MI355X (BASELINE.json configs[4]): StefCal
solve_gaintable core for 512 stations x 256 channels x 1000 times = 256,000
per-(time, channel) solves (B jones), run in batches of 16 gain rows
(4096 sub-solves).  True gains g = lognormal(0, 0.1) exp(i N(0, 0.1)) per
batch (seeded, generated on device), x_b = g_a1 conj(g_a2), unit weights;
the timed region is the batched solve (kernels.solve_gains) of every batch;
input generation is reported separately."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
import numpy as np, torch
from ska_sdp_func_python_amd import kernels

nants, nchan, ntime, batch = 512, 256, int(sys.argv[1]) if len(sys.argv) > 1 else 1000, 16
dev = torch.device("cuda:0")
a1, a2 = np.triu_indices(nants, 1)
perm, conj, rs, ant2 = kernels.canonical_baselines(a1, a2, nants)
a1t = torch.as_tensor(a1[perm], device=dev)
a2t = torch.as_tensor(a2[perm], device=dev)
gen = torch.Generator(device=dev)
gen.manual_seed(1805550721)
t_solve = t_gen = 0.0
iters, worst_err, worst_res = [], 0.0, 0.0
for t0 in range(0, ntime, batch):
    nt = min(batch, ntime - t0)
    torch.cuda.synchronize(); ta = time.perf_counter()
    amp = torch.exp(0.1 * torch.randn((nt, nants, nchan), generator=gen, device=dev, dtype=torch.float64))
    ph = 0.1 * torch.randn((nt, nants, nchan), generator=gen, device=dev, dtype=torch.float64)
    g = torch.polar(amp, ph)
    xb = (g[:, a1t, :] * torch.conj(g[:, a2t, :]))[..., None].contiguous()
    wb = torch.ones(xb.shape, dtype=torch.float64, device=dev)
    gain = torch.ones((nt, nants, nchan, 1, 1), dtype=torch.complex128, device=dev)
    gwt = torch.zeros((nt, nants, nchan, 1, 1), dtype=torch.float64, device=dev)
    torch.cuda.synchronize(); tb = time.perf_counter()
    res, used = kernels.solve_gains(xb, wb, gain, gwt, rs, ant2, mode=0, niter=200, tol=1e-6,
                                    phase_only=False)
    torch.cuda.synchronize(); tc = time.perf_counter()
    t_gen += tb - ta
    t_solve += tc - tb
    iters.append(int(used.max()))
    # gains are determined up to one phase per (time, chan): compare after
    # referencing both to antenna 0
    est = gain[..., 0, 0]
    est = est * torch.conj(est[:, :1]) / torch.abs(est[:, :1])
    tru = g * torch.conj(g[:, :1]) / torch.abs(g[:, :1])
    worst_err = max(worst_err, float(torch.max(torch.abs(est - tru))))
    worst_res = max(worst_res, float(res.max()))
    del xb, wb, g, gain, gwt
    if t0 % 160 == 0:
        print(f"rows {t0 + nt}/{ntime}: solve {t_solve:.2f} s", flush=True)
nsub = ntime * nchan
nbl = len(a1)
print(json.dumps({"path": "C5 StefCal (B jones) 512 st x 256 chan x %d times" % ntime,
                  "sub_solves": nsub, "solve_s": round(t_solve, 3), "gen_s": round(t_gen, 3),
                  "solves_per_s": round(nsub / t_solve, 1), "iterations_max": max(iters),
                  "iterations_median": int(np.median(iters)),
                  "max_gain_err": worst_err, "max_residual": worst_res,
                  # CPU port: 0.24 s per 512-station sub-solve (ref_oracle.stefcal_row,
                  # 1 core; scripts/bench_paths.py stefcal leg)
                  "cpu_estimate_h": round(nsub * 0.24 / 3600, 1)}), flush=True)
