"""GPU parity of the convolution-function gridder/degridder
(sdp_hip_grid_cf / sdp_hip_degrid_cf) and the centred FFTs against the
reference's own grid_visibility_to_griddata / degrid_visibility_from_griddata
/ fft / ifft outputs (tests/golden/cfgrid_*.npz, fft_centred.npz).  fp64
throughout: rtol 1e-10."""

import numpy as np
import pytest

from conftest import golden
from gpu_helpers import vis_from_arrays

pytestmark = pytest.mark.gpu


def _objects(g):
    from ska_sdp_func_python_amd import datamodels as dm
    pf = dm.PolarisationFrame(str(g["pol_frame"]))
    vis = vis_from_arrays(g["uvw"], g["freq"], g["vis"], weight=g["weight"], flags=g["flags"],
                          pf=pf.type)
    vis["imaging_weight"] = g["imaging_weight"]
    gw = dm.WCS(4, ["UU", "VV", "STOKES", "FREQ"], list(g["grid_crpix"]), list(g["grid_cdelt"]),
                list(g["grid_crval"]))
    cw = dm.WCS(7, ["UU", "VV", "DUU", "DVV", "WW", "STOKES", "FREQ"], list(g["cf_crpix"]),
                list(g["cf_cdelt"]), list(g["cf_crval"]))
    gd = dm.GridData.constructor(np.zeros(g["grid"].shape, complex), gw, pf)
    cf = dm.ConvolutionFunction.constructor(g["cf"], cw, pf)
    return vis, gd, cf


@pytest.mark.parametrize("tag", ["p1", "p4"])
def test_grid_degrid_match_reference(tag):
    from ska_sdp_func_python_amd.grid_data import (degrid_visibility_from_griddata,
                                                   grid_visibility_to_griddata)
    g = golden(f"cfgrid_{tag}.npz")
    vis, gd, cf = _objects(g)
    out, sumwt = grid_visibility_to_griddata(vis, gd, cf)
    np.testing.assert_allclose(out["pixels"].data, g["grid"], rtol=1e-10, atol=1e-9)
    np.testing.assert_allclose(sumwt, g["sumwt"], rtol=1e-12)
    gd2 = gd.copy(deep=True)
    gd2["pixels"].data = g["grid_in"]
    dv = degrid_visibility_from_griddata(vis, gd2, cf)
    np.testing.assert_allclose(dv.vis.data, g["degridded"], rtol=1e-10, atol=1e-9)


def test_centred_ffts_match_reference():
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.grid_data import fft_griddata_to_image, fft_image_to_griddata
    g = golden("fft_centred.npz")
    pf = dm.PolarisationFrame("stokesI")
    gd = dm.GridData.constructor(g["a"], dm.WCS(4), pf)
    tmpl = dm.create_image(32, 1e-3, dm.SkyCoord(0.0, 0.0))
    im = fft_griddata_to_image(gd, tmpl)
    np.testing.assert_allclose(im["pixels"].data, g["ifft"] * 32 * 32, rtol=1e-10, atol=1e-9)
    img = dm.Image.constructor(g["a"], pf, tmpl.image_acc.wcs)
    gd2 = fft_image_to_griddata(img, dm.GridData.constructor(np.zeros_like(g["a"]), dm.WCS(4), pf))
    np.testing.assert_allclose(gd2["pixels"].data, g["fft"], rtol=1e-10, atol=1e-9)


CHANNEL_MAPS = [(2, [0, 0], 1), (4, [0, 1, 1, 2], 3), (3, [2, -1, 0], 3)]


# CF supports: 64 taps (one per lane), non-square 60, 144 (two taps per
# lane), and 66 x 66 whose LDS tile (81^2 fp64 complex) exceeds 64 KiB, so it
# runs on the per-entry atomic kernel k_grid_cf
SUPPORTS = [(8, 8, 64, 48), (10, 6, 64, 48), (12, 12, 64, 48), (66, 66, 160, 176)]


@pytest.mark.parametrize("gv,gu,ny,nx", SUPPORTS)
@pytest.mark.parametrize("nchan,v2i,gn", CHANNEL_MAPS)
def test_grid_cf_weights_and_skips_many_blocks(nchan, v2i, gn, gv, gu, ny, nx):
    """Many workgroups (the weight / skip partial-sum slots wrap, tiles split
    into several work items) with rows on the grid edge: grid, sumwt and the
    skipped-sample count against the restated reference loop
    (oracle/ref_oracle.grid_cf) and its edge rule; several image channels
    with a non-trivial vis->image channel map (a negative index counts from
    the end, as numpy does in the reference)."""
    import torch
    import ref_oracle as ro
    from ska_sdp_func_python_amd import kernels
    rng = np.random.default_rng(11)
    nrow, npol, nw, ndv, ndu = (9000 if gv < 20 else 1500), 2, 3, 4, 4
    maps_h = {"pu": rng.integers(-2, nx + 2, (nchan, nrow)), "pv": rng.integers(-2, ny + 2, (nchan, nrow)),
              "pwc": rng.integers(0, nw, (nchan, nrow)), "pdu": rng.integers(0, ndu, (nchan, nrow)),
              "pdv": rng.integers(0, ndv, (nchan, nrow))}
    vis = rng.normal(size=(nrow, nchan, npol)) + 1j * rng.normal(size=(nrow, nchan, npol))
    wt = rng.uniform(0.5, 2.0, (nrow, nchan, npol))
    cf = rng.normal(size=(gn, npol, nw, ndv, ndu, gv, gu)) + 1j * rng.normal(size=(gn, npol, nw, ndv, ndu, gv, gu))
    v2i = np.array(v2i)
    eg, esw = ro.grid_cf(maps_h, v2i, vis, wt, cf, (gn, npol, ny, nx))
    ok = ~((maps_h["pv"] - gv // 2 < 0) | (maps_h["pv"] + gv // 2 >= ny)
           | (maps_h["pu"] - gu // 2 < 0) | (maps_h["pu"] + gu // 2 >= nx))
    dev = torch.device("cuda:0")
    T = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
    maps = {k: T(v, torch.int32) for k, v in maps_h.items()}
    grid = torch.zeros((gn, npol, ny, nx), dtype=torch.complex128, device=dev)
    sumwt = torch.zeros((gn, npol), dtype=torch.float64, device=dev)
    skipped = kernels.grid_cf(maps, T(v2i, torch.int32), T(vis, torch.complex128),
                              T(wt, torch.float64), T(cf, torch.complex128), grid, sumwt)
    np.testing.assert_allclose(grid.cpu().numpy(), eg, rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(sumwt.cpu().numpy(), esw, rtol=1e-12)
    assert int(skipped.item()) == int((~ok).sum()) * npol
    assert 0 < (~ok).sum() and ok.sum() > 0


@pytest.mark.parametrize("nchan,v2i,gn", CHANNEL_MAPS)
def test_degrid_cf_skips_many_blocks(nchan, v2i, gn):
    """Degridding over many workgroups with rows on the grid edge: the
    visibilities against the restated reference loop (ref_oracle.degrid_cf;
    skipped samples are written as zero) and the skipped-sample count
    from the partial-sum slots, over several image channels."""
    import torch
    import ref_oracle as ro
    from ska_sdp_func_python_amd import kernels
    rng = np.random.default_rng(12)
    nrow, npol, ny, nx, gv, gu, nw, ndv, ndu = 9000, 2, 64, 48, 8, 8, 3, 4, 4
    maps_h = {"pu": rng.integers(-2, nx + 2, (nchan, nrow)), "pv": rng.integers(-2, ny + 2, (nchan, nrow)),
              "pwc": rng.integers(0, nw, (nchan, nrow)), "pdu": rng.integers(0, ndu, (nchan, nrow)),
              "pdv": rng.integers(0, ndv, (nchan, nrow))}
    grid_h = rng.normal(size=(gn, npol, ny, nx)) + 1j * rng.normal(size=(gn, npol, ny, nx))
    cf = rng.normal(size=(gn, npol, nw, ndv, ndu, gv, gu)) + 1j * rng.normal(size=(gn, npol, nw, ndv, ndu, gv, gu))
    v2i = np.array(v2i)
    ev = ro.degrid_cf(maps_h, v2i, grid_h, cf, nrow, nchan)
    ok = ~((maps_h["pv"] - gv // 2 < 0) | (maps_h["pv"] + gv // 2 >= ny)
           | (maps_h["pu"] - gu // 2 < 0) | (maps_h["pu"] + gu // 2 >= nx))
    dev = torch.device("cuda:0")
    T = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
    maps = {k: T(v, torch.int32) for k, v in maps_h.items()}
    out = torch.full((nrow, nchan, npol), 7.0 + 0j, dtype=torch.complex128, device=dev)
    skipped = kernels.degrid_cf(maps, T(v2i, torch.int32), T(grid_h, torch.complex128),
                                T(cf, torch.complex128), nrow, nchan, out)
    np.testing.assert_allclose(out.cpu().numpy(), ev, rtol=1e-10, atol=1e-10)
    assert int(skipped.item()) == int((~ok).sum()) * npol
    assert 0 < (~ok).sum() and ok.sum() > 0


def _aw_objects(g):
    from ska_sdp_func_python_amd import datamodels as dm
    vpf, ipf = dm.PolarisationFrame(str(g["vis_pf"])), dm.PolarisationFrame(str(g["im_pf"]))
    freq = g["freq"]
    vis_pc = dm.SkyCoord(*g["vis_pc"])
    im_pc = dm.SkyCoord(*g["im_pc"])
    vis = vis_from_arrays(g["uvw"], freq, g["vis"], weight=g["weight"], flags=g["flags"],
                          pf=vpf.type, phasecentre=vis_pc)
    vis["imaging_weight"] = g["imaging_weight"].copy()
    nchan = len(freq)
    mk = lambda pf: dm.create_image(int(g["npix"]), float(g["cell"]), im_pc, polarisation_frame=pf,
                                    frequency=float(freq[0]), channel_bandwidth=2e6, nchan=nchan)
    im = mk(ipf)
    gcf = mk(vpf)
    gcf["pixels"].data[...] = g["gcf"]
    cw = dm.WCS(7, ["UU", "VV", "DUU", "DVV", "WW", "STOKES", "FREQ"], list(g["cf_crpix"]),
                list(g["cf_cdelt"]), list(g["cf_crval"]))
    cf = dm.ConvolutionFunction.constructor(g["cf"], cw, vpf)
    return vis, im, (lambda _m: (gcf, cf)), im_pc


@pytest.mark.parametrize("tag", ["p1", "p4"])
def test_awprojection_matches_reference(tag):
    """invert_awprojection (dirty + PSF) and predict_awprojection against the
    reference's own wrappers (imaging/base.py:158-259, exec'd with its
    gridding / FFT / pol-image / phase-rotation helpers by make_golden.py),
    with the visibility phase centre offset from the image's so both
    directions of shift_vis_to_image's tangent-plane rotation run.  fp64
    throughout: rtol 1e-10."""
    from ska_sdp_func_python_amd.imaging import invert_visibility, predict_visibility
    g = golden(f"awproj_{tag}.npz")
    vis, im, gcfcf, im_pc = _aw_objects(g)
    vis0 = np.array(vis.vis.data, copy=True)
    dirty, sumwt = invert_visibility(vis, im, context="awprojection", gcfcf=gcfcf)
    np.testing.assert_allclose(sumwt, g["sumwt"], rtol=1e-12)
    np.testing.assert_allclose(np.asarray(dirty["pixels"].data), g["dirty"], rtol=1e-10,
                               atol=1e-10 * np.abs(g["dirty"]).max())
    np.testing.assert_array_equal(np.asarray(vis.vis.data), vis0)  # input untouched
    psf, psw = invert_visibility(vis, im, dopsf=True, context="awprojection", gcfcf=gcfcf)
    np.testing.assert_allclose(psw, g["psf_sumwt"], rtol=1e-12)
    np.testing.assert_allclose(np.asarray(psf["pixels"].data), g["psf"], rtol=1e-10,
                               atol=1e-10 * np.abs(g["psf"]).max())
    model = im.copy(deep=True)
    model["pixels"].data = g["model"].copy()
    pv = predict_visibility(vis, model, context="awprojection", gcfcf=gcfcf)
    np.testing.assert_allclose(np.asarray(pv.vis.data), g["predicted"], rtol=1e-10,
                               atol=1e-10 * np.abs(g["predicted"]).max())
    assert pv.phasecentre.separation(im_pc).rad < 1e-12
    with pytest.raises(ValueError, match="gcfcf not specified"):
        invert_visibility(vis, im, context="awprojection")
