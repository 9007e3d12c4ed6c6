"""Builders shared by the GPU tests (fixture arrays -> datamodels shim objects)."""

import numpy as np

from ska_sdp_func_python_amd import datamodels as dm


def vis_from_arrays(uvw, freq, vis, weight=None, flags=None, baselines=None, pf="stokesI",
                    times=None, phasecentre=None, integration_time=None):
    nt, nb = uvw.shape[:2]
    if baselines is None:
        baselines = np.stack(np.triu_indices(64, 1), 1)[:nb]
    shape = vis.shape
    times = np.arange(nt, dtype=float) if times is None else times
    return dm.Visibility.constructor(
        frequency=np.asarray(freq, float), channel_bandwidth=np.full(len(freq), 1e6),
        phasecentre=phasecentre or dm.SkyCoord(0.0, -0.8), uvw=uvw, time=times,
        vis=vis, weight=np.ones(shape) if weight is None else weight,
        flags=np.zeros(shape, int) if flags is None else flags, baselines=baselines,
        polarisation_frame=dm.PolarisationFrame(pf), integration_time=integration_time)


def exact_pixels_dev(uvw, freqs, vis, npix, cell, px, py, rows=2_000_000):
    """The exact direct sum of ms2dirty (ducc0 convention with w-stacking,
    oracle/nufft_oracle.ms2dirty_exact; unit weights) at pixels (px[i],
    py[i]) in fp64 on the device: torch restatement for the full-size tests,
    whose 10^10 visibilities the CPU oracle sums only at a few pixels.
    ``uvw`` [nrow, 3] device f64 in the ducc0 frame (flips applied), ``freqs``
    uniformly spaced (numpy), ``vis`` [nrow, nchan] device complex.  The
    channel phasors follow exp(2 pi i t f_c) = exp(2 pi i t f_0) exp(2 pi i t
    df)^c in fp64 (oracle/wgrid_cpu.c row_phasors does the same).  Returns
    numpy f64 [len(px)]."""
    import math
    import torch
    freqs = np.asarray(freqs, dtype=float)
    if freqs.size > 1:
        df = np.diff(freqs)
        assert np.allclose(df, df[0], rtol=1e-9, atol=0.0), "uniform channels only"
    dev = uvw.device
    x = (torch.as_tensor(np.asarray(px), device=dev, dtype=torch.float64) - npix // 2) * cell
    y = (torch.as_tensor(np.asarray(py), device=dev, dtype=torch.float64) - npix // 2) * cell
    r2 = x * x + y * y
    nm1 = -r2 / (torch.sqrt(1.0 - r2) + 1.0)
    f0 = float(freqs[0])
    dfc = float(freqs[1] - freqs[0]) if freqs.size > 1 else 0.0
    out = torch.zeros(x.shape[0], dtype=torch.float64, device=dev)
    c = 299792458.0
    for a in range(0, uvw.shape[0], rows):
        u = uvw[a:a + rows]
        t = (u[:, 0:1] * x[None, :] + u[:, 1:2] * y[None, :] - u[:, 2:3] * nm1[None, :]) / c
        ph = torch.polar(torch.ones_like(t), 2.0 * math.pi * torch.remainder(t * f0, 1.0))
        st = torch.polar(torch.ones_like(t), 2.0 * math.pi * torch.remainder(t * dfc, 1.0))
        v = vis[a:a + rows].to(torch.complex128)
        for ch in range(freqs.size):
            out += (v[:, ch:ch + 1] * ph).real.sum(0)
            ph = ph * st
    inside = r2 < 1.0
    return torch.where(inside, out / (nm1 + 1.0), torch.zeros_like(out)).cpu().numpy()
