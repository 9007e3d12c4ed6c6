"""Measurement of the non-metric §8 rows on MI355X, each beside its CPU path.

One JSON line per path (SURVEY.md §8(d) work formulas):

* dft      C3: 1000 point components x 10 Mvis (19,306 baselines x 518 times,
           1 channel, stokesI). VALU bound; flops = N_vis N_comp (6 + 8 npol).
           CPU: the reference's dft_cpu_looped restated (oracle/ref_oracle.py)
           on a 100-component x 200k-visibility sample, scaled linearly.
* stefcal  C5-shaped batch: 512 stations, 64 times x 64 channels (B jones).
           HBM bound; 12 B per baseline per sub-solve iteration.
           CPU: the restated numpy solver (ref_oracle.stefcal_row) on 2
           sub-solves, scaled linearly.
* predict  C2 dirty2ms (4096^2 image, 8192^2 grid). Same roofline as invert.
           CPU: oracle/wgrid_cpu.c's dirty2ms (C + OpenMP restatement; ducc0
           absent) on 8 of the 64 channels: degridding scaled to the full
           visibility count, per-plane FFT + screen counted once.
* cfgrid   AW-projection gridding (grid_visibility_to_griddata kernel):
           4096^2 grid, 8x8 CF taps, 8x8 oversampling, 5 w planes, 4 Mvis,
           stokesI. fp64 global atomics (2 per tap).
           CPU: the reference's per-visibility loop restated (ref_oracle.grid_cf)
           on 30000 visibilities, scaled linearly.
* weighting C2 layout (123.6 Mvis, weight f64 + flags int64, the datamodels'
           dtypes) on the 4096^2 uv grid of the C2 image: weight_visibility
           uniform = grid_weights + reweight.  HBM bound; algorithmic bytes
           per sample: grid pass 8 (weight) + 8 (flags) + 24/nchan (uvw),
           reweight pass the same + 8 (imaging weight out).
           CPU: oracle/weighting_oracle.py (vectorised numpy restatement) on
           8 of the 64 channels, scaled linearly.
* calops   C5-shaped chunk: 512 stations (130,816 baselines), 16 times x 64
           channels, stokesI, c128 vis + model, f64 weight, int64 flags.
           point_sums (divide_visibility + solve_gaintable's per-row sums,
           B jones: one gain row per time) and apply_gaintable (forward).
           HBM bound: point_sums reads 16+16+8+8 B per sample; apply reads
           16+8 and writes 16+8 B per sample.
           CPU: oracle/calops_oracle.py (vectorised numpy) on 1 time, scaled.
"""

import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ska_sdp_func_python_amd import kernels, simulation  # noqa: E402

HBM_PEAK_GBS = 8000.0
FP32_PEAK_TFLOPS = 157.3
dev = torch.device("cuda:0")
which = (sys.argv[1].split(",") if len(sys.argv) > 1
         else ["dft", "stefcal", "predict", "cfgrid", "weighting", "calops"])
CORES = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0)),
            len(os.sched_getaffinity(0)))


def gpu_time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), r


def predict_cpu(obs, img, cell, nvis_full, nsample=8):
    """oracle/wgrid_cpu.c dirty2ms on nsample of the C2 channels (the extremes
    included, so the w planes match), scaled to the full job."""
    import wgrid_cpu
    nchan = obs["freq"].shape[0]
    chans = np.linspace(0, nchan - 1, nsample).round().astype(int)
    uvw = obs["uvw"].cpu().numpy().reshape(-1, 3) * np.array([-1.0, 1.0, -1.0])
    freq = obs["freq"].cpu().numpy()[chans]
    wgt = obs["wgt"].reshape(uvw.shape[0], nchan)[:, chans].cpu().numpy()
    t0 = time.perf_counter()
    _, tg, tf = wgrid_cpu.dirty2ms(uvw, freq, img.cpu().numpy(), wgt, cell, cell, 1e-12, True,
                                   nthreads=CORES)
    wall = time.perf_counter() - t0
    ns = uvw.shape[0] * nsample
    t_full = (wall - tf) * nvis_full / ns + tf
    return {"value": round(nvis_full / t_full / 1e6, 4), "unit": "Mvis/s", "cores": CORES,
            "kind": "port",
            "sample": (f"oracle/wgrid_cpu.c dirty2ms on {nsample} of {nchan} C2 channels "
                       f"({ns / 1e6:.2f} Mvis, same planes): {wall:.1f} s wall, of which "
                       f"{tf:.1f} s FFT+screen; degridding scaled by {nvis_full / ns:.0f}x")}


def emit(d):
    print(json.dumps(d), flush=True)


if "dft" in which:
    import ref_oracle as ro
    rng = np.random.default_rng(3)
    fn_, n_def, lat, dec = simulation.CONFIGS["MID"]
    ha = np.linspace(-0.5, 0.5, 518) * 8.0 * math.pi / 12.0
    uvw_h, _ = simulation.observe(fn_(n_def, seed=1), math.radians(lat), math.radians(dec), ha)
    uvw_h = uvw_h.reshape(-1, 3)
    uvw = torch.as_tensor(uvw_h, device=dev)
    freq_h = np.array([1.4e9])
    freq = torch.as_tensor(freq_h, device=dev)
    ncomp = 1000
    lm = rng.uniform(-0.05, 0.05, (ncomp, 2))
    dc_h = np.concatenate([lm, (np.sqrt(1 - (lm ** 2).sum(1)) - 1)[:, None]], 1)
    fl_h = rng.uniform(0.1, 10, (ncomp, 1, 1)).astype(complex)
    dc, fl = torch.as_tensor(dc_h, device=dev), torch.as_tensor(fl_h, device=dev)
    out = torch.empty((uvw.shape[0], 1, 1), dtype=torch.complex64, device=dev)
    t, _ = gpu_time(lambda: kernels.dft_point(dc, fl, uvw, freq=freq, out=out))
    nvis = uvw.shape[0]
    flops = nvis * ncomp * (6 + 8 * 1)
    # CPU sample: 100 components x 200k visibilities
    ns, nc = 200000, 100
    uvwl = uvw_h[:ns, None, :] * (freq_h / 299792458.0)[None, :, None]
    t0 = time.perf_counter()
    ro.dft_cpu_looped(dc_h[:nc], uvwl, fl_h[:nc])
    tc = time.perf_counter() - t0
    cpu_rate = ns * nc / tc
    emit({"path": "dft_skycomponent_visibility (C3)", "nvis": nvis, "ncomp": ncomp,
          "gpu_ms": round(t * 1e3, 3), "value": round(nvis * ncomp / t / 1e9, 2),
          "unit": "G comp*vis/s",
          "roofline": {"bound": "valu", "achieved": round(flops / t / 1e12, 2),
                       "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                       "frac": round(flops / t / 1e12 / FP32_PEAK_TFLOPS, 4),
                       "note": "flops = N_vis N_comp (6 + 8 npol), SURVEY.md 8(d); sincos excluded"},
          "cpu_baseline": {"value": round(cpu_rate / 1e9, 5), "unit": "G comp*vis/s", "cores": 1,
                           "kind": "port",
                           "sample": f"ref_oracle.dft_cpu_looped, {nc} comps x {ns} vis "
                                     f"({tc:.1f} s), numpy; full C3 extrapolates to "
                                     f"{nvis * ncomp / cpu_rate:.0f} s"}})
    del uvw, out

if "stefcal" in which:
    import ref_oracle as ro
    nants, nchan, ntime = 512, 64, 64
    a1, a2 = np.triu_indices(nants, 1)
    rng = np.random.default_rng(1805550721)
    g = (rng.lognormal(0, 0.1, (ntime, nants, nchan))
         * np.exp(1j * rng.normal(0, 0.1, (ntime, nants, nchan))))
    perm, conj, rs, ant2 = kernels.canonical_baselines(a1, a2, nants)
    gt = torch.as_tensor(g, device=dev)
    a1t, a2t = torch.as_tensor(a1[perm], device=dev), torch.as_tensor(a2[perm], device=dev)
    xb = (gt[:, a1t, :] * torch.conj(gt[:, a2t, :]))[..., None].contiguous()
    wb = torch.ones(xb.shape, dtype=torch.float64, device=dev)
    del gt

    def run():
        gain = torch.ones((ntime, nants, nchan, 1, 1), dtype=torch.complex128, device=dev)
        gwt = torch.zeros((ntime, nants, nchan, 1, 1), dtype=torch.float64, device=dev)
        return kernels.solve_gains(xb, wb, gain, gwt, rs, ant2, mode=0, niter=200, tol=1e-6,
                                   phase_only=False)
    t, (res, used) = gpu_time(run, reps=3)
    nsub = ntime * nchan
    iters = int(used.max())
    nbl = len(a1)
    gbs = 12 * nbl * nsub * iters / t / 1e9
    # CPU: the restated numpy solver on 2 single-channel sub-solves
    gh = g[:2, :, :1]
    bl = np.stack([a1, a2], 1)
    t0 = time.perf_counter()
    for s in range(2):
        xbh = (gh[s, a1] * np.conj(gh[s, a2]))[..., None]
        ro.stefcal_row(xbh, np.ones(xbh.shape), bl, nants, np.ones((nants, 1, 1, 1), complex),
                       np.zeros((nants, 1, 1, 1)), 200, 1e-6, False)
    tc = (time.perf_counter() - t0) / 2
    emit({"path": "solve_gaintable StefCal (C5-shaped batch)", "nants": nants,
          "sub_solves": nsub, "iterations": iters, "gpu_ms": round(t * 1e3, 3),
          "value": round(nsub / t, 1), "unit": "sub-solves/s",
          "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                       "note": "12 B per baseline per sub-solve iteration (c64 x + f32 w), "
                               "over the whole solve incl. k_fill / k_residual; k_iter alone: "
                               "profiles/r01_stefcal_kernel_stats.txt"},
          "max_residual": float(res.max()),
          "cpu_baseline": {"value": round(1.0 / tc, 2), "unit": "sub-solves/s", "cores": 1,
                           "kind": "port",
                           "sample": f"ref_oracle.stefcal_row (numpy), 2 sub-solves of 512 "
                                     f"stations, {tc:.2f} s each; C5 (256,000 sub-solves) "
                                     f"extrapolates to {256000 * tc / 3600:.1f} h"}})
    del xb, wb

if "predict" in which:
    obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, device=dev)
    cell = 0.25 / obs["umax"]
    img = torch.randn(4096, 4096, dtype=torch.float64, device=dev)
    out = torch.empty_like(obs["vis"])
    t, _ = gpu_time(lambda: kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell,
                                             1e-12, True, flip_uw=True, out=out))
    kernels.set_stage_timing(True)
    _, info = kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell, 1e-12, True,
                               flip_uw=True, out=out)
    kernels.set_stage_timing(False)
    nvis = obs["nrow"] * 64
    alg = nvis * (8 + 4 + 24.0 / 64) + info["nplanes"] * info["ngrid_x"] * info["ngrid_y"] * 8
    gbs = alg / (info["ms_grid"] * 1e-3) / 1e9
    emit({"path": "predict_ng / dirty2ms (C2)", "nvis": nvis, "gpu_ms": round(t * 1e3, 3),
          "value": round(nvis / t / 1e6, 1), "unit": "Mvis/s",
          "stages_ms": {k: round(info[k], 3) for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")},
          "roofline": {"bound": "hbm", "kernel": "k_degrid_mfma<8,true> (one-cell buckets)" if os.environ.get("SDP_HIP_MFMA_DEGRID", "1") != "0" else "k_degrid_reg<8,true>", "achieved": round(gbs, 1),
                       "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)},
          "cpu_baseline": predict_cpu(obs, img, cell, nvis)})
    del obs, img, out

if "cfgrid" in which:
    import ref_oracle as ro
    rng = np.random.default_rng(5)
    nrow, nchan, npol = 4_000_000, 1, 1
    ny = nx = 4096
    gv = gu = 8
    nw, ndv, ndu = 5, 8, 8
    maps_h = {"pu": rng.integers(gu, nx - gu, (nchan, nrow)), "pv": rng.integers(gv, ny - gv, (nchan, nrow)),
              "pwc": rng.integers(0, nw, (nchan, nrow)), "pdu": rng.integers(0, ndu, (nchan, nrow)),
              "pdv": rng.integers(0, ndv, (nchan, nrow))}
    maps = {k: torch.as_tensor(v.astype(np.int32), device=dev) for k, v in maps_h.items()}
    v2i = torch.zeros(nchan, dtype=torch.int32, device=dev)
    vis = torch.randn((nrow, nchan, npol), dtype=torch.complex128, device=dev)
    wt = torch.ones((nrow, nchan, npol), dtype=torch.float64, device=dev)
    cf_h = (rng.normal(size=(1, npol, nw, ndv, ndu, gv, gu))
            + 1j * rng.normal(size=(1, npol, nw, ndv, ndu, gv, gu)))
    cf = torch.as_tensor(cf_h, device=dev)
    grid = torch.zeros((1, npol, ny, nx), dtype=torch.complex128, device=dev)
    sumwt = torch.zeros((1, npol), dtype=torch.float64, device=dev)

    def run():
        grid.zero_()
        sumwt.zero_()
        return kernels.grid_cf(maps, v2i, vis, wt, cf, grid, sumwt)
    t, _ = gpu_time(run)
    # bytes: vis c128 + wt f64 + 5 int32 maps in, 2 fp64 atomics per tap out
    byts = nrow * (16 + 8 + 20) + nrow * gv * gu * 16
    gbs = byts / t / 1e9
    ns = 30000
    hm = {k: v[:, :ns] for k, v in maps_h.items()}
    vh = (rng.normal(size=(ns, nchan, npol)) + 1j * rng.normal(size=(ns, nchan, npol)))
    t0 = time.perf_counter()
    ro.grid_cf(hm, np.zeros(nchan, int), vh, np.ones((ns, nchan, npol)), cf_h, (1, npol, ny, nx))
    tc = time.perf_counter() - t0
    emit({"path": "grid_visibility_to_griddata (AW-projection CF gridding)", "nvis": nrow,
          "grid": f"{ny}x{nx}", "cf_taps": gv * gu, "gpu_ms": round(t * 1e3, 3),
          "value": round(nrow / t / 1e6, 1), "unit": "Mvis/s",
          "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                       "note": "the per-tap algorithm's bytes: inputs + 16 B (one complex add) per tap; the LDS tile turns the adds into one fp64 atomic per touched cell per work item"},
          "cpu_baseline": {"value": round(ns / tc / 1e6, 4), "unit": "Mvis/s", "cores": 1,
                           "kind": "port",
                           "sample": f"ref_oracle.grid_cf (the reference's per-visibility loop), "
                                     f"{ns} vis in {tc:.1f} s"}})

if "weighting" in which:
    import weighting_oracle as wo
    nchan = 64
    obs = simulation.device_observation(100, nchan, 0.95e9, 1.76e9, device=dev)
    nrow = obs["nrow"]
    uvw, freq = obs["uvw"].contiguous(), obs["freq"]
    del obs
    torch.manual_seed(3)
    wt = torch.rand((nrow, nchan, 1), dtype=torch.float64, device=dev) + 0.5
    flags = (torch.rand((nrow, nchan, 1), device=dev) < 0.01).to(torch.int64)
    iw = torch.empty_like(wt)
    freq_h = freq.cpu().numpy()
    uvw_h = uvw.cpu().numpy()
    umax = float(np.abs(uvw_h[:, :2]).max() * freq_h.max() / wo.C_M_S)
    n = 4096
    cell = 0.25 / umax
    du = 1.0 / (n * cell)
    wcs = ((0.0, -du, n // 2 + 1), (0.0, du, n // 2 + 1))
    v2i = torch.zeros(nchan, dtype=torch.int32, device=dev)
    grid = torch.zeros((1, 1, n, n), dtype=torch.float64, device=dev)
    sumwt = torch.zeros((1, 1), dtype=torch.float64, device=dev)

    def gridw():
        grid.zero_()
        sumwt.zero_()
        return kernels.grid_weights(uvw, freq, wt, flags, v2i, wcs, grid, sumwt)

    t_grid, sk = gpu_time(gridw)
    t_uni, _ = gpu_time(lambda: kernels.reweight(uvw, freq, wt, flags, v2i, wcs, grid, iw, "uniform"))
    t_rob, _ = gpu_time(lambda: kernels.reweight(uvw, freq, wt, flags, v2i, wcs, grid, iw, "robust",
                                                 robustness=0.0, sumwt=sumwt))
    t_tap, _ = gpu_time(lambda: kernels.taper(uvw, freq, flags, iw, "gaussian", 1e-6))
    nvis = nrow * nchan
    b_grid = nvis * (8 + 8 + 24.0 / nchan)
    b_rew = nvis * (8 + 8 + 8 + 24.0 / nchan)
    t_wv = t_grid + t_uni
    # CPU: 8-channel sample through the numpy restatement
    cs = 8
    sel = np.arange(cs) * (nchan // cs)
    wt_h = wt[:, sel].cpu().numpy()
    fl_h = flags[:, sel].cpu().numpy()
    t0 = time.perf_counter()
    g_h, s_h, _ = wo.grid_weights(uvw_h, freq_h[sel], wt_h * (1 - fl_h), np.zeros(cs, int), wcs, 1, n, n)
    wo.reweight(uvw_h, freq_h[sel], wt_h * (1 - fl_h), wt_h * (1 - fl_h), np.zeros(cs, int), wcs, g_h,
                "uniform")
    tc = (time.perf_counter() - t0) * nchan / cs
    emit({"path": "weight_visibility uniform (C2 layout, 4096^2 uv grid)", "nvis": nvis,
          "gpu_ms": round(t_wv * 1e3, 3), "value": round(nvis / t_wv / 1e6, 1), "unit": "Mvis/s",
          "stages_ms": {"grid_weights": round(t_grid * 1e3, 3), "reweight_uniform": round(t_uni * 1e3, 3),
                        "reweight_robust": round(t_rob * 1e3, 3), "taper_gaussian": round(t_tap * 1e3, 3)},
          "skipped": int(sk.item()),
          "roofline": {"bound": "hbm", "grid_weights_GBs": round(b_grid / t_grid / 1e9, 1),
                       "reweight_GBs": round(b_rew / t_uni / 1e9, 1), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round((b_grid + b_rew) / t_wv / 1e9 / HBM_PEAK_GBS, 4),
                       "note": "16.4 B/sample in (weight f64, flags int64, uvw), +8 B out for reweight"},
          "cpu_baseline": {"value": round(nvis / tc / 1e6, 3), "unit": "Mvis/s", "cores": 1,
                           "kind": "port",
                           "sample": f"weighting_oracle grid_weights + reweight (numpy) on {cs} of "
                                     f"{nchan} channels, {tc * cs / nchan:.1f} s, scaled x{nchan // cs}"}})

if "calops" in which:
    import calops_oracle as co
    nants, ntimes, nchan = 512, 16, 64
    a1, a2 = np.triu_indices(nants, 1)
    nbl = len(a1)
    shape = (ntimes, nbl, nchan, 1)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    v = torch.randn(shape, dtype=torch.complex128, device=dev, generator=g)
    m = torch.randn(shape, dtype=torch.complex128, device=dev, generator=g)
    w = torch.rand(shape, dtype=torch.float64, device=dev, generator=g) + 0.5
    f = (torch.rand(shape, device=dev, generator=g) < 0.01).to(torch.int64)
    ptr = torch.arange(ntimes + 1, dtype=torch.int32, device=dev)
    tidx = torch.arange(ntimes, dtype=torch.int32, device=dev)
    perm, conj, _, _ = kernels.canonical_baselines(a1, a2, nants)
    perm_d = torch.as_tensor(np.asarray(perm, np.int32), device=dev)
    conj_d = torch.as_tensor(np.asarray(conj, np.uint8), device=dev)
    t_ps, _ = gpu_time(lambda: kernels.point_sums(v, m, w, f, ptr, tidx, nchan, perm=perm_d,
                                                  conj=conj_d))
    gain = (torch.randn((ntimes, nants, nchan, 1, 1), dtype=torch.complex128, device=dev,
                        generator=g) + 2.0)
    a1d = torch.as_tensor(a1.astype(np.int32), device=dev)
    a2d = torch.as_tensor(a2.astype(np.int32), device=dev)
    trow = torch.arange(ntimes, dtype=torch.int32, device=dev)
    vv, ww = v.clone(), w.clone()
    t_ap, _ = gpu_time(lambda: kernels.apply_gains(vv, ww, None, False, a1d, a2d, trow, gain, False))
    nsamp = ntimes * nbl * nchan
    b_ps, b_ap = nsamp * 48, nsamp * 48
    # CPU: the numpy restatements on one time slot
    vh, mh, wh, fh = (x[:1].cpu().numpy() for x in (v, m, w, f))
    t0 = time.perf_counter()
    co.point_sums(vh, wh, fh, np.zeros(1), np.zeros(1), np.ones(1), nchan, model=mh)
    tc_ps = (time.perf_counter() - t0) * ntimes
    gh = gain[:1].cpu().numpy()
    t0 = time.perf_counter()
    co.apply_gaintable(vh, wh, fh, np.zeros(1), np.stack([a1, a2], 1), gh, np.zeros(1), np.ones(1))
    tc_ap = (time.perf_counter() - t0) * ntimes
    emit({"path": "calibration neighbours: point_sums (divide_visibility + x_b sums) and "
                  "apply_gaintable, 512 stations x 16 times x 64 chans", "nsamples": nsamp,
          "stages_ms": {"point_sums": round(t_ps * 1e3, 3), "apply_gaintable": round(t_ap * 1e3, 3)},
          "value": round(nsamp / t_ps / 1e9, 2), "unit": "Gsamples/s (point_sums)",
          "roofline": {"bound": "hbm", "point_sums_GBs": round(b_ps / t_ps / 1e9, 1),
                       "apply_GBs": round(b_ap / t_ap / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(b_ps / t_ps / 1e9 / HBM_PEAK_GBS, 4)},
          "cpu_baseline": {"value": round(nsamp / tc_ps / 1e9, 4), "unit": "Gsamples/s (point_sums)",
                           "apply_s": round(tc_ap, 2), "cores": 1, "kind": "port",
                           "sample": f"calops_oracle (numpy) on 1 of {ntimes} times, scaled"}})
