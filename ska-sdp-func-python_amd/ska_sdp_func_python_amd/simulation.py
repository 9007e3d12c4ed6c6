"""Seeded synthetic SKA-MID / SKA-LOW-like observations.

The datamodels antenna tables (create_named_configuration) are not available,
so layouts are generated: a dense core plus three logarithmic spiral arms,
sized like the real arrays (MID: 197 dishes, ~150 km max baseline;
LOW: 512 stations, ~74 km).  uvw follow the reference's ``xyz_to_uvw``
(util/coordinate_support.py:335-363) over an hour-angle range.
"""

import math

import numpy as np

from .datamodels import (PolarisationFrame, SkyCoord, Visibility)
from .util.coordinate_support import xyz_to_uvw

C = 299792458.0


def _spiral(rng, n, r_min, r_max, narms=3, twist=1.2):
    arm = np.arange(n) % narms
    t = np.sort(rng.uniform(0.0, 1.0, n))
    r = r_min * (r_max / r_min) ** t
    th = 2 * math.pi * arm / narms + twist * np.log(r / r_min) + rng.normal(0, 0.05, n)
    return np.stack([r * np.cos(th), r * np.sin(th)], 1)


def _disc(rng, n, r_max, power=0.5):
    r = r_max * rng.uniform(0, 1, n) ** power
    th = rng.uniform(0, 2 * math.pi, n)
    return np.stack([r * np.cos(th), r * np.sin(th)], 1)


def ska_mid_layout(ndish=197, seed=1):
    """(east, north) metres: 133 SKA dishes + 64 MeerKAT-like dishes."""
    rng = np.random.default_rng(seed)
    n_mk = min(64, ndish)
    n_ska = ndish - n_mk
    mk = np.concatenate([_disc(rng, min(48, n_mk), 1000.0), _disc(rng, n_mk - min(48, n_mk), 4000.0)])
    n_core = int(round(n_ska * 0.53))
    ska = np.concatenate([_disc(rng, n_core, 1200.0, 0.6), _spiral(rng, n_ska - n_core, 2000.0, 75000.0)])
    return np.concatenate([mk, ska])[:ndish]


def ska_low_layout(nstation=512, seed=2):
    """(east, north) metres: 224 core stations + clusters on 3 arms to ~37 km."""
    rng = np.random.default_rng(seed)
    n_core = min(224, nstation)
    core = _disc(rng, n_core, 500.0)
    n_out = nstation - n_core
    ncl = max(1, n_out // 8)
    centres = _spiral(rng, ncl, 1000.0, 37000.0)
    outer = np.concatenate([c + _disc(rng, 8, 100.0) for c in centres])[:n_out]
    if len(outer) < n_out:
        outer = np.concatenate([outer, _disc(rng, n_out - len(outer), 37000.0)])
    return np.concatenate([core, outer])[:nstation]


def enu_to_xyz(en, latitude):
    e, n = en[:, 0], en[:, 1]
    u = np.zeros_like(e)
    x = -math.sin(latitude) * n + math.cos(latitude) * u
    y = e
    z = math.cos(latitude) * n + math.sin(latitude) * u
    return np.stack([x, y, z], 1)


def baselines(nants, autos=False):
    a1, a2 = np.triu_indices(nants, 0 if autos else 1)
    return np.stack([a1, a2], 1)


def observe(layout_en, latitude, dec, times_ha, autos=False):
    """uvw [ntimes, nbl, 3] metres and the baseline list."""
    xyz = enu_to_xyz(layout_en, latitude)
    bl = baselines(len(xyz), autos)
    d = xyz[bl[:, 1]] - xyz[bl[:, 0]]
    uvw = np.stack([xyz_to_uvw(d, ha, dec) for ha in times_ha])
    return uvw, bl


CONFIGS = {
    # name: (layout fn, n, latitude deg, dec deg, nchan, f_lo, f_hi, ntimes, ha span hours)
    "MID": (ska_mid_layout, 197, -30.7, -45.0),
    "LOW": (ska_low_layout, 512, -26.8, -27.0),
}


def make_visibility(config="MID", nants=None, ntimes=10, nchan=1, f_lo=1.4e9, f_hi=None,
                    ha_span_h=2.0, dec_deg=None, polarisation_frame="stokesI", seed=0,
                    autos=False, phasecentre=None):
    """A synthetic Visibility (numpy arrays, unit weights, zero vis)."""
    fn, n_def, lat, dec_def = CONFIGS[config]
    n = nants or n_def
    lat = math.radians(lat)
    dec = math.radians(dec_deg if dec_deg is not None else dec_def)
    en = fn(n_def, seed=1 if config == "MID" else 2)[:n]
    ha = np.linspace(-0.5, 0.5, ntimes) * ha_span_h * math.pi / 12.0 if ntimes > 1 else np.zeros(1)
    uvw, bl = observe(en, lat, dec, ha, autos)
    freq = np.array([f_lo]) if nchan == 1 else np.linspace(f_lo, f_hi or f_lo * 1.25, nchan)
    bw = np.full(nchan, (freq[1] - freq[0]) if nchan > 1 else 1e6)
    pf = PolarisationFrame(polarisation_frame)
    shape = (ntimes, len(bl), nchan, pf.npol)
    pc = phasecentre or SkyCoord(0.0, dec)
    times = ha * 43200.0 / math.pi
    return Visibility.constructor(
        frequency=freq, channel_bandwidth=bw, phasecentre=pc, configuration=config,
        uvw=uvw, time=times, vis=np.zeros(shape, complex), weight=np.ones(shape),
        integration_time=np.full(ntimes, (times[1] - times[0]) if ntimes > 1 else 1.0),
        flags=np.zeros(shape, int), baselines=bl, polarisation_frame=pf)


def max_uv_lambda(vis):
    uvw = np.asarray(vis.uvw.data)
    fmax = float(np.max(vis.frequency.data))
    return float(np.max(np.abs(uvw[..., :2]))) * fmax / C


def c2_geometry(nchan=64, ntimes=100):
    """BASELINE.json configs[1]: SKA-MID 197 dishes, 64 chan x 100 times, 4096^2."""
    return dict(config="MID", ntimes=ntimes, nchan=nchan, f_lo=0.95e9, f_hi=1.76e9,
                ha_span_h=8.0, npix=4096)


def device_observation(ntimes, nchan, f_lo, f_hi, config="MID", ha_span_h=8.0, dec_deg=None,
                       seed=0, device=None, vis_dtype=None, chan_offset=0, nchan_total=None,
                       channels=None):
    """Device-resident C2/C4-style arrays without a host Visibility.

    Returns dict(uvw [nrow,3] f64, freq [nchan] f64, vis [nrow,nchan] c64,
    wgt [nrow,nchan] f32, nrow) generated on the GPU (seeded).  With
    ``chan_offset``/``nchan_total`` the channels are a slice of a wider band
    (one shard of a channel-sharded observation); ``channels`` instead picks
    explicit indices of the ``nchan_total`` band (interleaved shards).
    """
    import torch
    fn, n_def, lat, dec_def = CONFIGS[config]
    lat = math.radians(lat)
    dec = math.radians(dec_deg if dec_deg is not None else dec_def)
    en = fn(n_def, seed=1 if config == "MID" else 2)
    ha = np.linspace(-0.5, 0.5, ntimes) * ha_span_h * math.pi / 12.0
    uvw, _ = observe(en, lat, dec, ha)
    nt = nchan_total or nchan
    allf = np.linspace(f_lo, f_hi, nt) if nt > 1 else np.array([f_lo])
    if channels is not None:
        freq = allf[np.asarray(channels)]
        nchan = len(freq)
    else:
        freq = allf[chan_offset:chan_offset + nchan]
    dev = device or torch.device("cuda")
    uvw_t = torch.as_tensor(uvw.reshape(-1, 3), device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + seed)
    nrow = uvw_t.shape[0]
    vis = torch.randn((nrow, nchan), generator=g, device=dev, dtype=vis_dtype or torch.complex64)
    wgt = torch.ones((nrow, nchan), device=dev, dtype=torch.float32)
    return dict(uvw=uvw_t, freq=torch.as_tensor(freq, device=dev), vis=vis, wgt=wgt, nrow=nrow,
                umax=float(np.max(np.abs(uvw[..., :2]))) * float(allf.max()) / C)
