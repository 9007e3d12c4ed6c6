"""GPU: the sky-model drivers skymodel_predict_calibrate /
skymodel_calibrate_invert over the HIP DFT, NUFFT and apply_gaintable,
against the composition of the pinned oracles: ref_oracle.dft_cpu_looped
(reference dft fixtures), nufft_oracle exact sums (the sums ducc0
approximates) and calops_oracle.apply_gaintable (reference fixtures), with
the reference driver's mask / primary-beam / normalisation steps restated
here.  The reference's own test (tests/sky_model/test_skymodel_imaging.py)
reads an HDF5 sky model; h5py is absent here, so the sky model is synthetic.
Tolerance: relative RMS 5e-6 (the NUFFT term)."""

import math

import numpy as np
import pytest

import calops_oracle as co
import nufft_oracle as orc
import ref_oracle as ro
from conftest import rel_rms

pytestmark = pytest.mark.gpu
FLIP_UW = np.array([-1.0, 1.0, -1.0])
TOL = 5e-6


def _setup(seed=3):
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd import simulation
    rng = np.random.default_rng(seed)
    pc = dm.SkyCoord(math.radians(15.0), math.radians(-45.0))
    vis = simulation.make_visibility("LOW", nants=24, ntimes=4, nchan=3, f_lo=1.0e8, f_hi=1.1e8,
                                     ha_span_h=1.0, phasecentre=pc)
    npix = 128
    cell = 0.5 / (2 * simulation.max_uv_lambda(vis))
    f = np.asarray(vis.frequency.data)
    im = dm.create_image(npix, cell, pc, frequency=float(f.mean()), channel_bandwidth=1e8)
    px = np.zeros((1, 1, npix, npix))
    for _ in range(6):
        px[0, 0, rng.integers(40, 88), rng.integers(40, 88)] = rng.uniform(0.5, 2.0)
    im["pixels"].data = px
    comps = []
    for _ in range(4):
        x, y = rng.uniform(30, 98, 2)
        d = dm.pixel_to_skycoord(x, y, im.image_acc.wcs, origin=1)
        comps.append(dm.SkyComponent(d, f, flux=rng.uniform(1, 3, (3, 1)),
                                     polarisation_frame=dm.PolarisationFrame("stokesI")))
    mask = im.copy(deep=True)
    mpx = np.ones((1, 1, npix, npix))
    mpx[..., :, :24] = 0.0
    mpx[..., 100:, :] = 0.5
    mask["pixels"].data = mpx
    gt = dm.create_gaintable_from_visibility(vis, jones_type="B")
    gt["gain"].data = (rng.normal(1.0, 0.1, gt["gain"].data.shape)
                       * np.exp(1j * rng.normal(0, 0.3, gt["gain"].data.shape)))
    sm = dm.SkyModel(image=im, components=comps, gaintable=gt, mask=mask)
    return vis, sm, cell


def _pb(im):
    """A Gaussian 'primary beam' image over the model image."""
    npix = im["pixels"].data.shape[-1]
    y, x = np.mgrid[:npix, :npix] - npix // 2
    beam = im.copy(deep=True)
    beam["pixels"].data = np.exp(-(x ** 2 + y ** 2) / (2 * 40.0 ** 2))[None, None]
    return beam


def _beam_fluxes(comps, beam_px, wcs):
    from ska_sdp_func_python_amd import datamodels as dm
    out = []
    for c in comps:
        x, y = dm.skycoord_to_pixel(c.direction, wcs, origin=1)
        ix, iy = int(round(float(x[0]))), int(round(float(y[0])))
        out.append(c.flux * beam_px[:, :, iy, ix])
    return out


def _expected_predict(vis, sm, cell, beam=None):
    from ska_sdp_func_python_amd.util.coordinate_support import skycoord_to_lmn
    f = np.asarray(vis.frequency.data)
    uvw = np.asarray(vis.uvw.data)
    fl = _beam_fluxes(sm.components, sm.mask["pixels"].data, sm.mask.image_acc.wcs)
    if beam is not None:
        bf = _beam_fluxes(sm.components, beam["pixels"].data, beam.image_acc.wcs)
        fl = [a * (b / c.flux) for a, b, c in zip(fl, bf, sm.components)]
    dc = []
    for c in sm.components:
        l, m, _ = skycoord_to_lmn(c.direction, vis.phasecentre)
        dc.append([l, m, math.sqrt(1 - l * l - m * m) - 1.0])
    uvw_lambda = uvw[..., None, :] * (f / orc.C_LIGHT)[None, None, :, None]
    v = ro.dft_cpu_looped(np.array(dc), uvw_lambda, np.array(fl).astype(complex))
    img = sm.image["pixels"].data[0, 0] * sm.mask["pixels"].data[0, 0]
    if beam is not None:
        img = img * beam["pixels"].data[0, 0]
    nt, nb = uvw.shape[:2]
    pv = orc.dirty2ms_exact(uvw.reshape(-1, 3) * FLIP_UW, f, img.T, None, cell, cell, True)
    return v + pv.reshape(nt, nb, len(f), 1)


@pytest.mark.parametrize("use_pb", [False, True])
def test_skymodel_predict_calibrate(use_pb):
    from ska_sdp_func_python_amd.sky_model import skymodel_predict_calibrate
    vis, sm, cell = _setup()
    beam = _pb(sm.image) if use_pb else None
    calls = []

    def get_pb(v, im):
        calls.append(v.vis.shape[0])
        return beam

    out = skymodel_predict_calibrate(vis, sm, context="ng", docal=True, inverse=True,
                                     get_pb=get_pb if use_pb else None)
    expect = _expected_predict(vis, sm, cell, beam)
    g = sm.gaintable
    expect, _ = co.apply_gaintable(expect, np.asarray(vis.weight.data), np.asarray(vis.flags.data),
                                   np.asarray(vis.time.data), np.asarray(vis.baselines.data),
                                   g["gain"].data, g.time.data, g.interval.data, inverse=True)
    assert rel_rms(out.vis.data, expect) < TOL
    if use_pb:
        assert calls == [1, 1, 1, 1]


@pytest.mark.parametrize("use_pb", [False, True])
def test_skymodel_calibrate_invert(use_pb):
    from ska_sdp_func_python_amd.sky_model import skymodel_calibrate_invert
    vis, sm, cell = _setup(seed=5)
    rng = np.random.default_rng(9)
    vis["vis"].data = rng.normal(size=vis.vis.shape) + 1j * rng.normal(size=vis.vis.shape)
    beam = _pb(sm.image) if use_pb else None
    g = sm.gaintable
    cal, _ = co.apply_gaintable(vis.vis.data, np.asarray(vis.weight.data), np.asarray(vis.flags.data),
                                np.asarray(vis.time.data), np.asarray(vis.baselines.data), g["gain"].data,
                                g.time.data, g.interval.data, inverse=False)
    f = np.asarray(vis.frequency.data)
    uvw = np.asarray(vis.uvw.data)
    npix = sm.image["pixels"].data.shape[-1]
    res = skymodel_calibrate_invert(vis, sm, context="ng", docal=True,
                                    get_pb=(lambda v, im: beam) if use_pb else None)
    mask = sm.mask["pixels"].data[0, 0]
    if not use_pb:
        d = orc.ms2dirty_exact(uvw.reshape(-1, 3) * FLIP_UW, f, cal.reshape(-1, len(f)), None, npix,
                               npix, cell, cell, True).T / cal[..., 0].size
        assert rel_rms(np.asarray(res[0]["pixels"].data)[0, 0], d * mask) < TOL
        return
    flat = mask * beam["pixels"].data[0, 0]
    sd = np.zeros((npix, npix))
    sf = np.zeros((npix, npix))
    for t in range(uvw.shape[0]):
        d = orc.ms2dirty_exact(uvw[t] * FLIP_UW, f, cal[t].reshape(-1, len(f)), None, npix, npix,
                               cell, cell, True).T
        sd += flat * d
        sf += flat * flat * cal[t][..., 0].size
    maxwt = sf.max()
    assert rel_rms(np.asarray(res[0]["pixels"].data)[0, 0], sd / maxwt) < TOL
    np.testing.assert_allclose(np.asarray(res[1]["pixels"].data)[0, 0], np.sqrt(np.sqrt(sf / maxwt)),
                               rtol=1e-12)
