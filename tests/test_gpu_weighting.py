"""GPU parity of the imaging-weight path through the
C ABI: weight gridding, uniform / robust / natural reweighting and the two
tapers, against the reference-generated fixtures (tests/golden/weight_*.npz,
rtol 1e-12: only the fp64 summation order differs) and, at larger sizes,
against the numpy restatement oracle/weighting_oracle.py (bit-exact with unit
weights, where every gridded value is an integer)."""

import math

import numpy as np
import pytest
import torch

import weighting_oracle as wo
from conftest import golden, weight_case

pytestmark = pytest.mark.gpu
RTOL = 1e-12


def _vis_from_fixture(g, c, device=False):
    from ska_sdp_func_python_amd import datamodels as dm
    nt, nb, nchan, npol = c["shape"]
    arrs = dict(uvw=g["uvw"], weight=g["weight"], flags=g["flags"],
                imaging_weight=g["imaging_weight"].copy(),
                vis=np.zeros(c["shape"], complex))
    if device:
        arrs = {k: torch.as_tensor(v, device="cuda") for k, v in arrs.items()}
        arrs["flags"] = arrs["flags"].to(torch.int32)
    return dm.Visibility.constructor(
        frequency=g["freq"], channel_bandwidth=np.full(nchan, 1e6), phasecentre=dm.SkyCoord(0, -0.5),
        time=np.arange(nt, dtype=float), baselines=np.stack(np.triu_indices(12, 1), 1)[:nb],
        polarisation_frame=c["pf"], **arrs)


def _np(x):
    return x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)


@pytest.mark.parametrize("device", [False, True])
@pytest.mark.parametrize("tag", ["p1", "p4"])
def test_weighting_matches_reference_fixture(tag, device):
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.grid_data import (grid_visibility_weight_to_griddata,
                                                   griddata_visibility_reweight)
    from ska_sdp_func_python_amd.imaging import (taper_visibility_gaussian,
                                                 taper_visibility_tukey, weight_visibility)
    g = golden(f"weight_{tag}.npz")
    c = weight_case(g)
    gd = dm.create_griddata_from_image(c["model"], polarisation_frame=c["pf"])
    gd, sumwt = grid_visibility_weight_to_griddata(_vis_from_fixture(g, c, device), gd)
    np.testing.assert_allclose(_np(gd["pixels"].data).real, g["grid"], rtol=RTOL, atol=1e-12)
    np.testing.assert_allclose(sumwt, g["sumwt"], rtol=RTOL)
    for key, kw in (("uniform", dict(weighting="uniform")),
                    ("robust0", dict(weighting="robust", robustness=0.0, sumwt=sumwt)),
                    ("robustm1p5", dict(weighting="robust", robustness=-1.5)),
                    ("natural", dict(weighting="natural"))):
        v = griddata_visibility_reweight(_vis_from_fixture(g, c, device),
                                         None if key == "natural" else gd, **kw)
        np.testing.assert_allclose(_np(v.imaging_weight.data), g[f"iw_{key}"], rtol=RTOL,
                                   err_msg=key)
    v = weight_visibility(_vis_from_fixture(g, c, device), c["model"], weighting="robust",
                          robustness=0.5)
    np.testing.assert_allclose(_np(v.imaging_weight.data), g["iw_wv_robust0p5"], rtol=RTOL)
    v = weight_visibility(_vis_from_fixture(g, c, device), c["model"], weighting="uniform")
    np.testing.assert_allclose(_np(v.imaging_weight.data), g["iw_wv_uniform"], rtol=RTOL)
    vg = taper_visibility_gaussian(v.copy(deep=True), beam=float(g["gauss_beam"]))
    np.testing.assert_allclose(_np(vg.imaging_weight.data), g["iw_gauss"], rtol=RTOL)
    vt = taper_visibility_tukey(v.copy(deep=True), tukey=float(g["tukey"]))
    np.testing.assert_allclose(_np(vt.imaging_weight.data), g["iw_tukey"], rtol=RTOL)


def _mid_case(ntimes, nchan, npol, seed, flag_frac=0.05, unit=True):
    from ska_sdp_func_python_amd import simulation
    fn, n_def, lat, dec = simulation.CONFIGS["MID"]
    ha = np.linspace(-0.5, 0.5, ntimes) * 8.0 * math.pi / 12.0
    uvw, _ = simulation.observe(fn(n_def, seed=1), math.radians(lat), math.radians(dec), ha)
    uvw = uvw.reshape(-1, 3)
    freq = np.linspace(0.95e9, 1.76e9, nchan)
    rng = np.random.default_rng(seed)
    shape = (uvw.shape[0], nchan, npol)
    wt = np.ones(shape) if unit else rng.uniform(0.5, 2.0, shape)
    flags = (rng.uniform(size=shape) < flag_frac).astype(np.int64)
    return uvw, freq, wt, flags


def _dev(*a):
    return [torch.as_tensor(np.ascontiguousarray(x), device="cuda") for x in a]


@pytest.mark.parametrize("npol,g_nchan,shift", [(1, 1, 0.0), (4, 2, 0.0), (1, 1, 0.37)])
def test_weight_grid_bit_exact_vs_oracle(npol, g_nchan, shift):
    """SKA-MID 197 dishes x 30 times x 16 channels on a 1024^2 uv grid sized so
    the longest baselines fall off it: unit weights make every gridded value
    an integer, so grid, sumwt, skip count and uniform weights are exact.
    shift != 0 moves crval off zero (no conjugate-mirror folding)."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, wt, flags = _mid_case(30, 16, npol, seed=3)
    umax = np.abs(uvw[:, :2]).max() * freq.max() / wo.C_M_S
    n = 1024
    du = 2 * 0.8 * umax / n
    wcs = ((shift * du, -du, n // 2 + 1), (-shift * du, du, n // 2 + 1))
    v2i = (np.arange(16) * g_nchan) // 16
    fwt = wt * (1 - flags)
    ref_grid, ref_sumwt, ref_skip = wo.grid_weights(uvw, freq, fwt, v2i, wcs, g_nchan, n, n)
    d_uvw, d_freq, d_wt, d_fl = _dev(uvw, freq, wt, flags)
    d_v2i = torch.as_tensor(v2i, dtype=torch.int32, device="cuda")
    grid = torch.zeros((g_nchan, npol, n, n), dtype=torch.float64, device="cuda")
    sumwt = torch.zeros((g_nchan, npol), dtype=torch.float64, device="cuda")
    skipped = kernels.grid_weights(d_uvw, d_freq, d_wt, d_fl, d_v2i, wcs, grid, sumwt)
    assert ref_skip > 0 and int(skipped.item()) == ref_skip
    assert np.array_equal(grid.cpu().numpy(), ref_grid)
    assert np.array_equal(sumwt.cpu().numpy(), ref_sumwt)
    imw = np.random.default_rng(5).uniform(0.5, 2.0, wt.shape)
    ref_iw = wo.reweight(uvw, freq, fwt, imw * (1 - flags), v2i, wcs, ref_grid, "uniform")
    d_iw = _dev(imw)[0]
    kernels.reweight(d_uvw, d_freq, d_wt, d_fl, d_v2i, wcs, grid, d_iw, "uniform")
    assert np.array_equal(d_iw.cpu().numpy(), ref_iw)
    for rob, sw in ((0.0, None), (-0.7, ref_sumwt)):
        ref_iw = wo.reweight(uvw, freq, fwt, imw * (1 - flags), v2i, wcs, ref_grid, "robust",
                             robustness=rob, sumwt=sw)
        d_iw = _dev(imw)[0]
        kernels.reweight(d_uvw, d_freq, d_wt, d_fl, d_v2i, wcs, grid, d_iw, "robust",
                         robustness=rob, sumwt=None if sw is None else _dev(sw)[0])
        np.testing.assert_allclose(d_iw.cpu().numpy(), ref_iw, rtol=RTOL)


def test_weighting_random_weights_and_tapers_vs_oracle():
    from ska_sdp_func_python_amd import kernels
    uvw, freq, wt, flags = _mid_case(20, 12, 2, seed=9, unit=False)
    flags = flags.astype(np.int8)
    umax = np.abs(uvw[:, :2]).max() * freq.max() / wo.C_M_S
    n = 512
    du = 2 * 1.1 * umax / n
    wcs = ((0.0, -du, n // 2 + 1), (0.0, du, n // 2 + 1))
    v2i = np.zeros(12, dtype=int)
    fwt = wt * (1 - flags)
    ref_grid, ref_sumwt, ref_skip = wo.grid_weights(uvw, freq, fwt, v2i, wcs, 1, n, n)
    d_uvw, d_freq, d_wt, d_fl = _dev(uvw, freq, wt, flags)
    d_v2i = torch.zeros(12, dtype=torch.int32, device="cuda")
    grid = torch.zeros((1, 2, n, n), dtype=torch.float64, device="cuda")
    sumwt = torch.zeros((1, 2), dtype=torch.float64, device="cuda")
    skipped = kernels.grid_weights(d_uvw, d_freq, d_wt, d_fl, d_v2i, wcs, grid, sumwt)
    assert ref_skip == 0 and int(skipped.item()) == 0
    np.testing.assert_allclose(grid.cpu().numpy(), ref_grid, rtol=RTOL, atol=1e-12)
    np.testing.assert_allclose(sumwt.cpu().numpy(), ref_sumwt, rtol=RTOL)
    imw = np.random.default_rng(6).uniform(0.5, 2.0, wt.shape)
    fimw = imw * (1 - flags)
    for kind, param, ref in (
            ("gaussian", math.pi ** 2 * 1e-4 ** 2 / (4 * math.log(2)),
             wo.taper_gaussian(uvw, freq, fimw, 1e-4)),
            ("tukey", 0.25, wo.taper_tukey(uvw, freq, fimw, 0.25))):
        d_iw = _dev(imw)[0]
        kernels.taper(d_uvw, d_freq, d_fl, d_iw, kind, param)
        # 0.5 (1 + cos) cancels near the taper's zero: absolute 1e-15 there
        np.testing.assert_allclose(d_iw.cpu().numpy(), ref, rtol=1e-13, atol=1e-15, err_msg=kind)


def test_weighting_edge_cases():
    """All samples flagged -> empty grid, zero imaging weights; NaN uvw maps to
    the centre cell (nan_to_num, gridding.py:53-55); nrow = 0 is a no-op."""
    from ska_sdp_func_python_amd import kernels
    uvw = np.array([[10.0, 20.0, 0.0], [np.nan, 5.0, 0.0], [1e300, 1.0, 0.0]])
    freq = np.array([1e9, 1.1e9])
    wt = np.ones((3, 2, 1))
    n = 16
    wcs = ((0.0, -10.0, n // 2 + 1), (0.0, 10.0, n // 2 + 1))
    v2i = np.zeros(2, dtype=int)
    for flags in (np.zeros((3, 2, 1), np.int64), np.ones((3, 2, 1), np.int64)):
        ref_grid, ref_sumwt, ref_skip = wo.grid_weights(uvw, freq, wt * (1 - flags), v2i, wcs, 1,
                                                        n, n)
        d = _dev(uvw, freq, wt, flags)
        d_v2i = torch.zeros(2, dtype=torch.int32, device="cuda")
        grid = torch.zeros((1, 1, n, n), dtype=torch.float64, device="cuda")
        sumwt = torch.zeros((1, 1), dtype=torch.float64, device="cuda")
        sk = kernels.grid_weights(*d, d_v2i, wcs, grid, sumwt)
        assert int(sk.item()) == ref_skip == 2
        assert np.array_equal(grid.cpu().numpy(), ref_grid)
        assert np.array_equal(sumwt.cpu().numpy(), ref_sumwt)
        iw = _dev(np.full((3, 2, 1), 7.0))[0]
        kernels.reweight(*d, d_v2i, wcs, grid, iw, "uniform")
        ref = wo.reweight(uvw, freq, wt * (1 - flags), np.full((3, 2, 1), 7.0) * (1 - flags), v2i,
                          wcs, ref_grid, "uniform")
        assert np.array_equal(iw.cpu().numpy(), ref)
    z = torch.zeros((0, 3), dtype=torch.float64, device="cuda")
    zw = torch.zeros((0, 2, 1), dtype=torch.float64, device="cuda")
    sk = kernels.grid_weights(z, _dev(freq)[0], zw, None, torch.zeros(2, dtype=torch.int32,
                              device="cuda"), wcs, grid, sumwt)
    assert int(sk.item()) == 0
    with pytest.raises(AssertionError):
        kernels.reweight(z, _dev(freq)[0], zw, None, None, wcs, grid, zw, "briggs")
