"""GPU parity of the HIP w-stacking NUFFT (sdp_hip_ms2dirty / sdp_hip_dirty2ms)
against the exact direct sums ducc0 approximates (oracle/nufft_oracle.py).

Tolerance: dirty-image / visibility RMS error relative to the RMS of the
exact result < 5e-6 (north star: < 1e-5) with the default epsilon (W = 8)."""

import numpy as np
import pytest
import torch

import nufft_oracle as orc
from conftest import golden, rel_rms
from gpu_helpers import vis_from_arrays

pytestmark = pytest.mark.gpu
TOL = 5e-6
FLIP_UW = np.array([-1.0, 1.0, -1.0])


def dev():
    return torch.device("cuda:0")


def T(a, dt=None):
    return torch.as_tensor(np.asarray(a), device=dev(), dtype=dt)


def _problem(seed, nrow=300, nchan=3, umax=2000.0, frac=0.45):
    rng = np.random.default_rng(seed)
    freq = np.linspace(1.0e9, 1.2e9, nchan)
    uvw = rng.uniform(-1, 1, (nrow, 3)) * umax * orc.C_LIGHT / freq.max()
    uvw[:, 2] *= 0.6
    ms = rng.normal(size=(nrow, nchan)) + 1j * rng.normal(size=(nrow, nchan))
    wgt = rng.uniform(0.5, 1.5, (nrow, nchan)).astype(np.float32)
    return uvw, freq, ms, wgt, frac / umax


@pytest.fixture(params=["fine", "fine1", "coarse"])
def bucket(request, monkeypatch):
    """Every bucketing: one-cell buckets (4-padded for the invert's MFMA
    gridder, plain for the MFMA degridder) from the two-level LDS-histogram
    sort (k_t_*, the invert's default at these sizes; forced for the predict
    too by SDP_HIP_BUCKET2=2), the same buckets from the single-level global
    histogram (SDP_HIP_BUCKET2=0, the fp32 predict's default), and 16x16-cell
    buckets sub-sorted by cell per work item (the path of very large grids
    such as C4's 16384^2 x 70 planes, forced here by SDP_HIP_BUCKET=16)."""
    if request.param == "fine":
        monkeypatch.setenv("SDP_HIP_BUCKET2", "2")
    if request.param == "coarse":
        monkeypatch.setenv("SDP_HIP_BUCKET", "16")
    if request.param == "fine1":
        monkeypatch.setenv("SDP_HIP_BUCKET2", "0")
    return request.param


@pytest.mark.parametrize("dow", [False, True])
@pytest.mark.parametrize("vdt", [torch.complex64, torch.complex128])
@pytest.mark.parametrize("flip", [False, True])
def test_ms2dirty_matches_exact(dow, vdt, flip, bucket):
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(1)
    npix = 64
    fl = np.array([-1.0, 1.0, -1.0]) if flip else np.ones(3)
    ex = orc.ms2dirty_exact(uvw * fl, freq, ms, wgt, npix, 48 + 16 * dow, cell, cell * 0.9, dow)
    out, info = kernels.ms2dirty(T(uvw), T(freq), T(ms, vdt), T(wgt), npix, 48 + 16 * dow, cell,
                                 cell * 0.9, 1e-7, dow, flip_uw=flip)
    assert info["support"] == 8
    assert info["bucket"] == (16 if bucket == "coarse" else 1)
    assert info["tiled"] == (1 if bucket == "fine" else 0)
    assert info["padded"] == 1  # invert: k_grid_mfma_pad on 4-padded cells
    assert info["grid_launches"] == 1
    assert rel_rms(out.cpu().numpy(), ex) < TOL


@pytest.mark.parametrize("dow", [False, True])
def test_dirty2ms_matches_exact(dow, bucket):
    from ska_sdp_func_python_amd import kernels
    uvw, freq, _, wgt, cell = _problem(2)
    rng = np.random.default_rng(5)
    img = rng.normal(size=(64, 64))
    ex = orc.dirty2ms_exact(uvw, freq, img, wgt, cell, cell, dow)
    for vdt in (torch.complex64, torch.complex128):
        v, _ = kernels.dirty2ms(T(uvw), T(freq), T(img), T(wgt), cell, cell, 1e-7, dow, vis_dtype=vdt)
        assert rel_rms(v.cpu().numpy(), ex) < TOL


def test_image_rows_not_a_multiple_of_4():
    """ny % 4 != 0 takes the 8-byte plane transposes (the 16-byte ones pair
    image rows across the ky wrap only when ny / 2 is even): invert and
    predict against the exact sums."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(6)
    ex = orc.ms2dirty_exact(uvw, freq, ms, wgt, 60, 50, cell, cell, True)
    out, _ = kernels.ms2dirty(T(uvw), T(freq), T(ms), T(wgt), 60, 50, cell, cell, 1e-7, True)
    assert rel_rms(out.cpu().numpy(), ex) < TOL
    img = np.random.default_rng(7).normal(size=(60, 50))
    exv = orc.dirty2ms_exact(uvw, freq, img, wgt, cell, cell, True)
    v, _ = kernels.dirty2ms(T(uvw), T(freq), T(img), T(wgt), cell, cell, 1e-7, True)
    assert rel_rms(v.cpu().numpy(), exv) < TOL


def test_unit_visibilities_weights_and_accumulate():
    """vis=None (PSF) and wgt=None are unit arrays; ACCUMULATE adds."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, _, _, cell = _problem(3)
    ones = np.ones((uvw.shape[0], len(freq)))
    ex = orc.ms2dirty_exact(uvw, freq, ones, None, 64, 64, cell, cell, True)
    out, _ = kernels.ms2dirty(T(uvw), T(freq), None, None, 64, 64, cell, cell, 1e-7, True)
    assert rel_rms(out.cpu().numpy(), ex) < TOL
    kernels.ms2dirty(T(uvw), T(freq), None, None, 64, 64, cell, cell, 1e-7, True, out=out,
                     accumulate=True)
    assert rel_rms(out.cpu().numpy(), 2 * ex) < TOL


def test_zero_weights_skip_and_psf_peak():
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(4)
    wgt[::3] = 0.0
    ex = orc.ms2dirty_exact(uvw, freq, ms, wgt, 64, 64, cell, cell, True)
    out, info = kernels.ms2dirty(T(uvw), T(freq), T(ms), T(wgt), 64, 64, cell, cell, 1e-7, True)
    assert info["nvis_used"] == int((wgt != 0).sum())
    assert rel_rms(out.cpu().numpy(), ex) < TOL
    psf, _ = kernels.ms2dirty(T(uvw), T(freq), None, T(wgt), 64, 64, cell, cell, 1e-7, True)
    psf = psf.cpu().numpy() / wgt.sum()
    assert abs(psf[32, 32] - 1.0) < 1e-6 and psf.max() <= psf[32, 32] + 1e-9


def test_nyquist_violation_raises():
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(5, frac=0.6)
    with pytest.raises(ValueError):
        kernels.ms2dirty(T(uvw), T(freq), T(ms), T(wgt), 64, 64, cell, cell, 1e-7, True)


@pytest.mark.parametrize("npix,nrow,nchan", [(1024, 20000, 16)])
def test_adjointness_at_scale(npix, nrow, nchan, bucket):
    """<A x, y> == <x, A^H y> for the w-stacked pair at a size the oracle cannot
    sum directly (size-independent property)."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(6, nrow=nrow, nchan=nchan, umax=2e4)
    rng = np.random.default_rng(7)
    img = rng.normal(size=(npix, npix))
    d, _ = kernels.ms2dirty(T(uvw), T(freq), T(ms), None, npix, npix, cell, cell, 1e-7, True)
    v, _ = kernels.dirty2ms(T(uvw), T(freq), T(img), None, cell, cell, 1e-7, True,
                            vis_dtype=torch.complex128)
    lhs = float(np.sum(d.cpu().numpy() * img))
    rhs = float(np.real(np.vdot(v.cpu().numpy(), ms)))  # Re sum conj(A img) . ms
    assert abs(lhs - rhs) / abs(lhs) < 1e-5


def test_linearity_at_scale(bucket):
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(8, nrow=30000, nchan=8, umax=2e4)
    a, _ = kernels.ms2dirty(T(uvw), T(freq), T(ms), T(wgt), 512, 512, cell, cell, 1e-7, True)
    b, _ = kernels.ms2dirty(T(uvw), T(freq), T(2.5 * ms), T(wgt), 512, 512, cell, cell, 1e-7, True)
    assert rel_rms(b.cpu().numpy(), 2.5 * a.cpu().numpy()) < 1e-6


def _c1_objects(g):
    from ska_sdp_func_python_amd import datamodels as dm
    uvw = g["uvw"].reshape(10, 21, 3)
    vis = vis_from_arrays(uvw, g["freq"], g["ms"].reshape(10, 21, 1, 1),
                          weight=g["wgt"].reshape(10, 21, 1, 1), phasecentre=dm.SkyCoord(0.0, -0.785))
    vis["imaging_weight"] = g["wgt"].reshape(10, 21, 1, 1).copy()
    im = dm.create_image(256, float(g["cell"]), dm.SkyCoord(0.0, -0.785), frequency=float(g["freq"][0]))
    return vis, im


@pytest.mark.parametrize("dow", [0, 1])
def test_invert_ng_c1_fixture(dow):
    """C1 (SKA-MID 7-dish subset, 10 times, 1 chan, 256^2) through the
    reference-shaped invert_ng: flips, transpose, sumwt normalisation."""
    from ska_sdp_func_python_amd.imaging import invert_ng
    g = golden("nufft_c1.npz")
    vis, im = _c1_objects(g)
    dirty, sumwt = invert_ng(vis, im, do_wstacking=bool(dow))
    np.testing.assert_allclose(sumwt, [[g["wgt"].sum()]], rtol=1e-6)
    expect = g[f"dirty_w{dow}"].T / g["wgt"].sum()
    assert rel_rms(dirty["pixels"].data[0, 0], expect) < TOL


@pytest.mark.parametrize("dow", [0, 1])
def test_predict_ng_c1_fixture(dow):
    from ska_sdp_func_python_amd.imaging import predict_ng
    g = golden("nufft_c1.npz")
    vis, im = _c1_objects(g)
    im["pixels"].data[0, 0] = g[f"model_w{dow}"].T
    pv = predict_ng(vis, im, do_wstacking=bool(dow))
    assert rel_rms(pv.vis.data.reshape(-1), g[f"vis_w{dow}"].reshape(-1)) < TOL


def test_context_2d_is_ng_without_wstacking():
    """reference imaging/imaging.py:46-55, :87-105: context "2d" is ng with
    do_wstacking=False -- checked against the C1 fixture's no-w-term exact
    results through invert_visibility / predict_visibility."""
    from ska_sdp_func_python_amd.imaging import invert_visibility, predict_visibility
    g = golden("nufft_c1.npz")
    vis, im = _c1_objects(g)
    dirty, sumwt = invert_visibility(vis, im, context="2d")
    expect = g["dirty_w0"].T / g["wgt"].sum()
    assert rel_rms(dirty["pixels"].data[0, 0], expect) < TOL
    assert rel_rms(dirty["pixels"].data[0, 0], g["dirty_w1"].T / g["wgt"].sum()) > 10 * TOL
    im["pixels"].data[0, 0] = g["model_w0"].T
    pv = predict_visibility(vis, im, context="2d")
    assert rel_rms(pv.vis.data.reshape(-1), g["vis_w0"].reshape(-1)) < TOL


def test_invert_predict_round_trip_point_source():
    """Reference property (tests/imaging/test_imaging.py:216-226): a unit
    point at the image centre predicts visibilities ~1."""
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd import simulation
    from ska_sdp_func_python_amd.imaging import invert_visibility, predict_visibility
    vis = simulation.make_visibility("MID", nants=20, ntimes=5, nchan=2, f_lo=1.4e9)
    cell = 0.5 / (2 * simulation.max_uv_lambda(vis))
    im = dm.create_image(256, cell, vis.phasecentre, frequency=1.4e9)
    im["pixels"].data[0, 0, 128, 128] = 1.0
    pv = predict_visibility(vis, im, context="ng")
    np.testing.assert_allclose(pv.vis.data, 1.0, atol=1e-5)
    psf, sw = invert_visibility(pv, im, dopsf=True, context="ng")
    assert abs(psf["pixels"].data[0, 0, 128, 128] - 1.0) < 1e-5


def test_plane_chunking_matches_resident(bucket, monkeypatch):
    """A grid budget of one plane forces plane-by-plane passes (the path very
    large grids take); results equal the all-planes-resident ones."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(9, nrow=3000, nchan=4, umax=4000.0)
    args = (T(uvw), T(freq), T(ms), T(wgt), 256, 256, cell, cell, 1e-7, True)
    full, info = kernels.ms2dirty(*args)
    img = torch.randn(256, 256, dtype=torch.float64, device=dev())
    vfull, _ = kernels.dirty2ms(T(uvw), T(freq), img, T(wgt), cell, cell, 1e-7, True,
                                vis_dtype=torch.complex128)
    monkeypatch.setenv("SDP_HIP_GRID_BUDGET_GB", "0.0001")
    part, info2 = kernels.ms2dirty(*args)
    vpart, _ = kernels.dirty2ms(T(uvw), T(freq), img, T(wgt), cell, cell, 1e-7, True,
                                vis_dtype=torch.complex128)
    assert info["nplanes"] > 2 and info2["plane_chunk"] == 1
    assert rel_rms(part.cpu().numpy(), full.cpu().numpy()) < 1e-6
    assert rel_rms(vpart.cpu().numpy(), vfull.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("fft_planes,budget", [("2", None), ("3", "0.002")])
def test_fft_batches_match_single_batch(fft_planes, budget, monkeypatch):
    """The per-plane FFT / w-screen stages run in batches of fft_planes planes
    (the y-spectra buffers of very large grids hold only a batch): batches of
    2 or 3 planes, with all planes resident or in plane chunks, equal one
    batch over all planes for both directions."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(10, nrow=3000, nchan=4, umax=4000.0)
    args = (T(uvw), T(freq), T(ms), T(wgt), 256, 256, cell, cell, 1e-7, True)
    img = torch.randn(256, 256, dtype=torch.float64, device=dev())
    full, info = kernels.ms2dirty(*args)
    vfull, _ = kernels.dirty2ms(T(uvw), T(freq), img, T(wgt), cell, cell, 1e-7, True,
                                vis_dtype=torch.complex128)
    monkeypatch.setenv("SDP_HIP_FFT_PLANES", fft_planes)
    if budget:
        monkeypatch.setenv("SDP_HIP_GRID_BUDGET_GB", budget)
    part, info2 = kernels.ms2dirty(*args)
    vpart, _ = kernels.dirty2ms(T(uvw), T(freq), img, T(wgt), cell, cell, 1e-7, True,
                                vis_dtype=torch.complex128)
    assert info["nplanes"] > 3
    assert rel_rms(part.cpu().numpy(), full.cpu().numpy()) < 1e-6
    assert rel_rms(vpart.cpu().numpy(), vfull.cpu().numpy()) < 1e-6


def test_large_grid_adjointness(monkeypatch):
    """C4-size grid (8192^2 image, 16384^2 grid, 2.15 GB planes) on the
    16x16-bucket path (MFMA kernels on cell-sub-sorted items):
    <A x, y> = <x, A^H y> and ms2dirty of the predicted visibilities of a
    point source peaks at that source."""
    from ska_sdp_func_python_amd import kernels
    monkeypatch.setenv("SDP_HIP_BUCKET", "16")
    npix = 8192
    uvw, freq, ms, _, _ = _problem(11, nrow=20000, nchan=4, umax=3.0e5)
    uvw[:, 2] *= 0.02  # a handful of w planes at this cell size
    cell = 0.45 / 3.0e5
    rng = np.random.default_rng(12)
    img = torch.zeros((npix, npix), dtype=torch.float64, device=dev())
    ix = rng.integers(npix // 4, 3 * npix // 4, 64)
    iy = rng.integers(npix // 4, 3 * npix // 4, 64)
    img[ix, iy] = torch.as_tensor(rng.normal(size=64), device=dev())
    d, info = kernels.ms2dirty(T(uvw), T(freq), T(ms), None, npix, npix, cell, cell, 1e-7, True)
    assert info["bucket"] == 16 and info["ngrid_x"] == 2 * npix and info["nplanes"] >= 8
    v, _ = kernels.dirty2ms(T(uvw), T(freq), img, None, cell, cell, 1e-7, True,
                            vis_dtype=torch.complex128)
    lhs = float(torch.sum(d * img))
    rhs = float(np.real(np.vdot(v.cpu().numpy(), ms)))
    assert abs(lhs - rhs) / abs(lhs) < 1e-5
    # a unit point source: predicted vis have |V| = 1 (exact phasors) and
    # the dirty image of them peaks at the source
    pt = torch.zeros_like(img)
    pt[int(ix[0]), int(iy[0])] = 1.0
    vp, _ = kernels.dirty2ms(T(uvw), T(freq), pt, None, cell, cell, 1e-7, True,
                             vis_dtype=torch.complex128)
    assert float(torch.max(torch.abs(torch.abs(vp) - 1.0))) < 1e-5
    dp, _ = kernels.ms2dirty(T(uvw), T(freq), vp, None, npix, npix, cell, cell, 1e-7, True)
    k = int(torch.argmax(dp))
    assert (k // npix, k % npix) == (int(ix[0]), int(iy[0]))


def test_full_size_invert_matches_c_restatement():
    """C2 geometry at the full 4096^2 image (8192^2 grid, 9 w planes): the HIP
    invert of 2 of the 64 channels against oracle/wgrid_cpu.c (the C
    restatement of the same w-gridding algorithm, itself pinned to the exact
    direct sums in tests/test_oracle_golden.py).  Both sides approximate the
    exact sum to ~1e-6, so they agree to that level."""
    import math
    import wgrid_cpu
    from ska_sdp_func_python_amd import kernels, simulation
    fn, n_def, lat, dec = simulation.CONFIGS["MID"]
    ha = np.linspace(-0.5, 0.5, 100) * 8.0 * math.pi / 12.0
    uvw, _ = simulation.observe(fn(n_def, seed=1), math.radians(lat), math.radians(dec), ha)
    uvw = uvw.reshape(-1, 3)
    allf = np.linspace(0.95e9, 1.76e9, 64)
    umax = float(np.max(np.abs(uvw[:, :2]))) * allf.max() / orc.C_LIGHT
    freq = allf[[0, 63]]
    rng = np.random.default_rng(17)
    ms = (rng.normal(size=(uvw.shape[0], 2)) + 1j * rng.normal(size=(uvw.shape[0], 2))).astype(np.complex64)
    cell = 0.25 / umax
    fuvw = uvw * FLIP_UW
    ref, _, _ = wgrid_cpu.ms2dirty(fuvw, freq, ms, None, 4096, 4096, cell, cell, 1e-12, True,
                                   nthreads=16)
    out, info = kernels.ms2dirty(T(uvw), T(freq), T(ms), None, 4096, 4096, cell, cell, 1e-7, True,
                                 flip_uw=True)
    assert info["nplanes"] >= 8 and info["ngrid_x"] == 8192
    assert rel_rms(out.cpu().numpy(), ref) < 5e-6



def test_full_size_predict_matches_c_restatement():
    """The predict counterpart of the test above: HIP dirty2ms of a random
    4096^2 image at 2 of the C2 channels against oracle/wgrid_cpu.c's dirty2ms
    (pinned to exact sums and to the C1 fixture on the CPU)."""
    import math
    import wgrid_cpu
    from ska_sdp_func_python_amd import kernels, simulation
    fn, n_def, lat, dec = simulation.CONFIGS["MID"]
    ha = np.linspace(-0.5, 0.5, 100) * 8.0 * math.pi / 12.0
    uvw, _ = simulation.observe(fn(n_def, seed=1), math.radians(lat), math.radians(dec), ha)
    uvw = uvw.reshape(-1, 3)
    allf = np.linspace(0.95e9, 1.76e9, 64)
    umax = float(np.max(np.abs(uvw[:, :2]))) * allf.max() / orc.C_LIGHT
    freq = allf[[0, 63]]
    rng = np.random.default_rng(18)
    img = rng.normal(size=(4096, 4096))
    wgt = rng.uniform(0.5, 1.5, (uvw.shape[0], 2)).astype(np.float32)
    cell = 0.25 / umax
    ref, _, _ = wgrid_cpu.dirty2ms(uvw * FLIP_UW, freq, img, wgt, cell, cell, 1e-12, True,
                                   nthreads=16)
    v, info = kernels.dirty2ms(T(uvw), T(freq), T(img), T(wgt), cell, cell, 1e-7, True,
                               flip_uw=True)
    assert info["nplanes"] >= 8 and info["ngrid_x"] == 8192
    assert rel_rms(v.cpu().numpy(), ref) < 5e-6

def _prologue_reference(vis, im, dopsf):
    """numpy restatement of invert_ng's visibility prologue (reference
    imaging/ng.py:191-204, :231-233): flagged vis -> image pol frame, flagged
    imaging weights; returns (ms [nrow, nchan, npol], wgt, uvw)."""
    from ska_sdp_func_python_amd import datamodels as dm
    nt, nb, nchan, npol = vis.vis.data.shape
    ms = (vis.vis.data * (1 - vis.flags.data)).reshape(nt * nb, nchan, npol)
    ms = dm.convert_pol_frame(ms, vis.visibility_acc.polarisation_frame,
                              im.image_acc.polarisation_frame, polaxis=2)
    wgt = (vis.imaging_weight.data * (1 - vis.flags.data)).reshape(nt * nb, nchan, npol)
    if dopsf:
        ms = np.zeros_like(ms)
        ms[..., 0] = 1.0
    return ms, wgt, vis.uvw.data.reshape(-1, 3)


@pytest.mark.parametrize("pf,ipf", [("stokesI", "stokesI"), ("linear", "stokesIQUV"),
                                    ("circular", "stokesIQUV"), ("linear", "linear")])
@pytest.mark.parametrize("mfs", [True, False])
@pytest.mark.parametrize("dopsf", [False, True])
@pytest.mark.parametrize("device", [False, True])
def test_invert_ng_fused_prologue(pf, ipf, mfs, dopsf, device):
    """invert_ng reads the Visibility in place through sdp_hip_ms2dirty_vis:
    flag masking of vis and weights, the pol-frame conversion, f64 weights
    and sumwt, against the numpy prologue + exact sums (tolerance TOL; sumwt
    rtol 1e-12).  Device-resident inputs use c64 vis, f32 weights, int32
    flags; host inputs the datamodels' c128 / f64 / int64."""
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.imaging import invert_ng
    rng = np.random.default_rng(21)
    nt, nb, nchan = 5, 40, 3
    npol = dm.PolarisationFrame(pf).npol
    freq = np.linspace(1.0e9, 1.1e9, nchan)
    umax = 1500.0
    uvw = rng.uniform(-1, 1, (nt, nb, 3)) * umax * orc.C_LIGHT / freq.max()
    uvw[..., 2] *= 0.5
    shape = (nt, nb, nchan, npol)
    v = rng.normal(size=shape) + 1j * rng.normal(size=shape)
    w = rng.uniform(0.5, 2.0, shape)
    fl = (rng.uniform(size=shape) < 0.15).astype(int)
    vis = vis_from_arrays(uvw, freq, v, weight=w, flags=fl, pf=pf,
                          phasecentre=dm.SkyCoord(0.0, -0.6))
    vis["imaging_weight"] = rng.uniform(0.5, 2.0, shape)
    npix, cell = 128, 0.4 / umax
    fc, bw = (float(freq.mean()), 1e9) if mfs else (float(freq[0]), float(freq[1] - freq[0]))
    im = dm.create_image(npix, cell, dm.SkyCoord(0.0, -0.6), polarisation_frame=dm.PolarisationFrame(ipf),
                         frequency=fc, channel_bandwidth=bw, nchan=1 if mfs else nchan)
    ms, wgt, fuvw = _prologue_reference(vis, im, dopsf)
    if device:
        for name, dt in (("vis", torch.complex64), ("imaging_weight", torch.float32),
                         ("flags", torch.int32)):
            vis[name] = torch.as_tensor(np.asarray(vis[name].data), device="cuda").to(dt)
        vis["uvw"] = torch.as_tensor(uvw, device="cuda")
    dirty, sumwt = invert_ng(vis, im, dopsf=dopsf, normalise=False)
    img = dirty["pixels"].data
    img = img.cpu().numpy() if isinstance(img, torch.Tensor) else img
    nimch = 1 if mfs else nchan
    exp_sw = np.zeros((nimch, npol))
    for pol in range(npol):
        for c in range(nimch):
            chans = slice(0, nchan) if mfs else slice(c, c + 1)
            exp_sw[c, pol] = wgt[:, chans, pol].sum()
            if dopsf and pol > 0:
                assert not np.any(img[c, pol])
                continue
            ref = orc.ms2dirty_exact(fuvw * FLIP_UW, freq[chans], ms[:, chans, pol],
                                     wgt[:, chans, pol], npix, npix, cell, cell, True).T
            assert rel_rms(img[c, pol], ref) < TOL, (pol, c)
    np.testing.assert_allclose(sumwt, exp_sw, rtol=1e-6 if device else 1e-12)


@pytest.mark.parametrize("eps,tol", [(1e-7, 1e-6), (1e-12, 1e-10)])
def test_invert_ng_host_visibility_streamed(eps, tol, monkeypatch):
    """A host-resident Visibility (numpy c128 / f64 / int64) is copied in time
    blocks, block k + 1 on a copy stream while block k grids, as one batch
    sequence through one set of w planes (SDP_HIP_HOST_BLOCKS, ragged blocks
    of 7 times): the same image as copying everything first (fp32 atomics'
    order only, or fp64) and the same sumwt, and the exact sums."""
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.imaging import invert_ng
    rng = np.random.default_rng(29)
    nt, nb, nchan = 7, 60, 4
    freq = np.linspace(1.0e9, 1.2e9, nchan)
    umax = 1500.0
    uvw = rng.uniform(-1, 1, (nt, nb, 3)) * umax * orc.C_LIGHT / freq.max()
    uvw[..., 2] *= 0.5
    shape = (nt, nb, nchan, 1)
    v = rng.normal(size=shape) + 1j * rng.normal(size=shape)
    fl = (rng.uniform(size=shape) < 0.1).astype(np.int64)
    vis = vis_from_arrays(uvw, freq, v, weight=rng.uniform(0.5, 2.0, shape), flags=fl,
                          pf="stokesI", phasecentre=dm.SkyCoord(0.0, -0.6))
    vis["imaging_weight"] = rng.uniform(0.5, 2.0, shape)
    npix, cell = 128, 0.4 / umax
    im = dm.create_image(npix, cell, dm.SkyCoord(0.0, -0.6), frequency=float(freq.mean()),
                         channel_bandwidth=1e9, nchan=1)
    out = {}
    for nblk in ("4", "1"):
        monkeypatch.setenv("SDP_HIP_HOST_BLOCKS", nblk)
        d, sw = invert_ng(vis, im, normalise=False, epsilon=eps)
        out[nblk] = (np.asarray(d["pixels"].data)[0, 0], sw)
    np.testing.assert_allclose(out["4"][1], out["1"][1], rtol=1e-13)
    assert rel_rms(out["4"][0], out["1"][0]) < tol
    ms, wgt, fuvw = _prologue_reference(vis, im, False)
    ref = orc.ms2dirty_exact(fuvw * FLIP_UW, freq, ms[..., 0], wgt[..., 0], npix, npix, cell,
                             cell, True).T
    assert rel_rms(out["4"][0], ref) < (TOL if eps > 1e-8 else 1e-9)


@pytest.mark.parametrize("eps", [1e-6, 1e-12])
def test_invert_ng_host_visibility_planes_chunked(eps, monkeypatch):
    """When the w planes cannot all stay resident (a grid budget of one plane,
    SDP_HIP_GRID_BUDGET_GB), a batch sequence cannot hold them, so the
    streamed host invert falls back to copying the Visibility whole and one
    call with chunked planes: the same image and sumwt as the resident
    call, and the exact sums."""
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.imaging import invert_ng
    rng = np.random.default_rng(31)
    nt, nb, nchan = 6, 50, 3
    freq = np.linspace(1.0e9, 1.2e9, nchan)
    umax = 1500.0
    uvw = rng.uniform(-1, 1, (nt, nb, 3)) * umax * orc.C_LIGHT / freq.max()
    shape = (nt, nb, nchan, 1)
    v = rng.normal(size=shape) + 1j * rng.normal(size=shape)
    vis = vis_from_arrays(uvw, freq, v, weight=rng.uniform(0.5, 2.0, shape),
                          pf="stokesI", phasecentre=dm.SkyCoord(0.0, -0.6))
    vis["imaging_weight"] = rng.uniform(0.5, 2.0, shape)
    npix, cell = 128, 0.4 / umax
    im = dm.create_image(npix, cell, dm.SkyCoord(0.0, -0.6), frequency=float(freq.mean()),
                         channel_bandwidth=1e9, nchan=1)
    monkeypatch.setenv("SDP_HIP_HOST_BLOCKS", "3")
    d0, sw0 = invert_ng(vis, im, normalise=False, epsilon=eps)
    monkeypatch.setenv("SDP_HIP_GRID_BUDGET_GB", "0.000001")
    d1, sw1 = invert_ng(vis, im, normalise=False, epsilon=eps)
    monkeypatch.delenv("SDP_HIP_GRID_BUDGET_GB")
    a0, a1 = np.asarray(d0["pixels"].data)[0, 0], np.asarray(d1["pixels"].data)[0, 0]
    np.testing.assert_allclose(sw1, sw0, rtol=1e-13)
    assert rel_rms(a1, a0) < (1e-6 if eps > 1e-8 else 1e-12)
    ms, wgt, fuvw = _prologue_reference(vis, im, False)
    ref = orc.ms2dirty_exact(fuvw * FLIP_UW, freq, ms[..., 0], wgt[..., 0], npix, npix, cell,
                             cell, True).T
    assert rel_rms(a1, ref) < (TOL if eps > 1e-8 else 1e-9)


@pytest.mark.parametrize("pf,ipf,dopsf", [("stokesI", "stokesI", False),
                                          ("linear", "stokesIQUV", True),
                                          ("linear", "stokesIQUV", False)])
@pytest.mark.parametrize("order", ["sorted", "interleaved"])
def test_invert_ng_cube_channel_runs(pf, ipf, dopsf, order, monkeypatch):
    """A cube whose image channels each collect several visibility channels
    (8 -> 2, the reference's many-to-one vis_to_im, ng.py:259-289): invert_ng
    grids each run of consecutive channels of one image channel as one call.
    With interleaved frequencies the runs alternate image channels, so two
    calls add into one image; the pipelined (two-stream) result must equal
    the one-stream result (SDP_HIP_OVERLAP=0) and the exact sums per image
    channel, and sumwt must count every channel once."""
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.imaging import invert_ng
    rng = np.random.default_rng(23)
    nt, nb, nchan = 6, 40, 8
    npol = dm.PolarisationFrame(pf).npol
    freq = 1.0e9 + 1.0e7 * np.arange(nchan)
    if order == "interleaved":
        freq = freq[[0, 4, 1, 5, 2, 6, 3, 7]]
    umax = 1500.0
    uvw = rng.uniform(-1, 1, (nt, nb, 3)) * umax * orc.C_LIGHT / freq.max()
    uvw[..., 2] *= 0.5
    shape = (nt, nb, nchan, npol)
    v = rng.normal(size=shape) + 1j * rng.normal(size=shape)
    fl = (rng.uniform(size=shape) < 0.1).astype(int)
    vis = vis_from_arrays(uvw, freq, v, weight=rng.uniform(0.5, 2.0, shape), flags=fl, pf=pf,
                          phasecentre=dm.SkyCoord(0.0, -0.6))
    vis["imaging_weight"] = rng.uniform(0.5, 2.0, shape)
    npix, cell = 128, 0.4 / umax
    im = dm.create_image(npix, cell, dm.SkyCoord(0.0, -0.6),
                         polarisation_frame=dm.PolarisationFrame(ipf), frequency=1.015e9,
                         channel_bandwidth=4.0e7, nchan=2)
    ichan = np.round((freq - 1.015e9) / 4.0e7).astype(int)
    assert sorted(np.bincount(ichan)) == [4, 4]
    ms, wgt, fuvw = _prologue_reference(vis, im, dopsf)
    out = {}
    for tag in ("1", "0"):
        monkeypatch.setenv("SDP_HIP_OVERLAP", tag)
        d, sw = invert_ng(vis, im, dopsf=dopsf, normalise=False)
        out[tag] = (np.asarray(d["pixels"].data), sw)
    np.testing.assert_allclose(out["1"][1], out["0"][1], rtol=1e-13)
    assert rel_rms(out["1"][0], out["0"][0]) < 1e-6  # fp32 atomics' order only
    for c in range(2):
        chans = np.flatnonzero(ichan == c)
        for pol in range(npol):
            np.testing.assert_allclose(out["1"][1][c, pol], wgt[:, chans, pol].sum(), rtol=1e-12)
            if dopsf and pol > 0:
                assert not np.any(out["1"][0][c, pol])
                continue
            ref = orc.ms2dirty_exact(fuvw * FLIP_UW, freq[chans], ms[:, chans, pol],
                                     wgt[:, chans, pol], npix, npix, cell, cell, True).T
            assert rel_rms(out["1"][0][c, pol], ref) < TOL, (c, pol)


@pytest.mark.parametrize("bucket2", ["1", "2"])
def test_shared_bucketing_across_pols(bucket2, monkeypatch):
    """SDP_HIP_KEEP_BUCKETS / SDP_HIP_REUSE_BUCKETS (invert_ng's image pols):
    pol 0 keeps its bucketing, pols 1-3 -- different weights and flags, pol 0
    zero where the others are not -- re-run only the value pass.  Each image
    and weight sum equals an independent call (1e-6 relative RMS: the order
    of the fp32 sums inside a cell differs; sumwt 1e-12); a reuse after
    another wstack call, or with other uvw, is refused.  A kept bucketing is
    single-level by default; SDP_HIP_BUCKET2=2 keeps a two-level one."""
    from ska_sdp_func_python_amd import kernels
    monkeypatch.setenv("SDP_HIP_BUCKET2", bucket2)
    rng = np.random.default_rng(71)
    nrow, nchan, npol, npix = 6000, 8, 4, 256
    freq = np.linspace(1.0e9, 1.2e9, nchan)
    umax = 3000.0
    uvw_h = rng.uniform(-1, 1, (nrow, 3)) * umax * orc.C_LIGHT / freq.max()
    uvw_h[:, 2] *= 0.3
    dev = "cuda"
    uvw = torch.as_tensor(uvw_h, device=dev)
    freq_t = torch.as_tensor(freq, device=dev)
    vis = torch.as_tensor(rng.normal(size=(nrow, nchan, npol)) +
                          1j * rng.normal(size=(nrow, nchan, npol)), device=dev).to(torch.complex64)
    flags = torch.as_tensor(rng.uniform(size=(nrow, nchan, npol)) < 0.2, device=dev).to(torch.int32)
    wgt = torch.as_tensor(rng.uniform(0.5, 2.0, (nrow, nchan, npol)), device=dev)
    wgt[: nrow // 3, :, 0] = 0.0  # pol 0 drops rows the other pols grid
    cell = 0.35 / umax
    args = (npix, npix, cell, cell, 1e-5, True)

    def run(pol, **kw):
        sw = torch.zeros(1, dtype=torch.float64, device=dev)
        out, info = kernels.ms2dirty_vis(uvw, freq_t, vis, pol, wgt[:, :, pol].contiguous(), flags,
                                         None, *args, flip_uw=True, sumwt=sw, **kw)
        return out.cpu().numpy(), float(sw.cpu()), info

    ind = [run(p) for p in range(npol)]
    shared = [run(0, keep_buckets=True)] + [run(p, reuse_buckets=True) for p in range(1, npol)]
    for p in range(npol):
        assert rel_rms(shared[p][0], ind[p][0]) < 1e-6, p
        assert abs(shared[p][1] - ind[p][1]) <= 1e-12 * abs(ind[p][1])
    assert shared[0][2]["nvis_used"] == nrow * nchan  # zero weights bucketed too
    assert shared[0][2]["tiled"] == (1 if bucket2 == "2" else 0)
    # any other wstack call drops the kept bucketing
    kernels.dirty2ms(uvw, freq_t, torch.zeros((npix, npix), dtype=torch.float64, device=dev),
                     None, cell, cell, 1e-5, True, flip_uw=True)
    with pytest.raises(ValueError, match="no kept bucketing"):
        run(1, reuse_buckets=True)
    run(0, keep_buckets=True)
    uvw2 = uvw.clone()
    with pytest.raises(ValueError, match="must be those of"):
        kernels.ms2dirty_vis(uvw2, freq_t, vis, 1, wgt[:, :, 1].contiguous(), flags, None, *args,
                             flip_uw=True, reuse_buckets=True)


@pytest.mark.parametrize("path", ["fused", "coarse", "fp64"])
@pytest.mark.parametrize("vdt", [torch.complex64, torch.complex128])
def test_pols_call_matches_per_pol_calls(path, vdt, monkeypatch):
    """sdp_hip_ms2dirty_vis_pols (invert_ng's image pols in one call: one
    bucketing, one value pass writing every pol's records) against one
    ms2dirty_vis call per image pol: a linear -> stokesIQUV conversion matrix,
    int8 flags, f64 weights that differ per pol (pol 0 zero on a third of the
    rows).  "coarse" (16x16-cell buckets) and "fp64" (epsilon 1e-12) are plans
    the fused pass does not cover: the library runs them pol by pol.  Images
    1e-6 relative RMS (fp32 sums inside a cell), weight sums 1e-12."""
    from ska_sdp_func_python_amd import kernels
    if path == "coarse":
        monkeypatch.setenv("SDP_HIP_BUCKET", "16")
    rng = np.random.default_rng(72)
    nrow, nchan, npv, npix = 5000, 6, 4, 128
    freq = np.linspace(1.0e9, 1.2e9, nchan)
    umax = 3000.0
    uvw_h = rng.uniform(-1, 1, (nrow, 3)) * umax * orc.C_LIGHT / freq.max()
    uvw_h[:, 2] *= 0.3
    dev = "cuda"
    uvw = torch.as_tensor(uvw_h, device=dev)
    freq_t = torch.as_tensor(freq, device=dev)
    vis = torch.as_tensor(rng.normal(size=(nrow, nchan, npv)) +
                          1j * rng.normal(size=(nrow, nchan, npv)), device=dev).to(vdt)
    flags = torch.as_tensor(rng.uniform(size=(nrow, nchan, npv)) < 0.2, device=dev).to(torch.int8)
    wgt = torch.as_tensor(rng.uniform(0.5, 2.0, (nrow, nchan, npv)), device=dev)
    wgt[: nrow // 3, :, 0] = 0.0
    conv = [[1, 0, 0, 1], [1, 0, 0, -1], [0, 1, 1, 0], [0, -1j, 1j, 0]]  # linear -> IQUV
    cell = 0.35 / umax
    eps = 1e-12 if path == "fp64" else 1e-5
    args = (npix, npix, cell, cell, eps, True)
    ind, sws = [], []
    for q in range(4):
        sw = torch.zeros(1, dtype=torch.float64, device=dev)
        out, _ = kernels.ms2dirty_vis(uvw, freq_t, vis, q, wgt[:, :, q].contiguous(), flags,
                                      conv[q], *args, flip_uw=True, sumwt=sw)
        ind.append(out.cpu().numpy())
        sws.append(float(sw.cpu()))
    sw4 = torch.zeros(4, dtype=torch.float64, device=dev)
    out4, info = kernels.ms2dirty_vis_pols(uvw, freq_t, vis, wgt, flags, conv, *args,
                                           flip_uw=True, sumwt=sw4)
    got, gsw = out4.cpu().numpy(), sw4.cpu().numpy()
    tol = 1e-12 if path == "fp64" else 1e-6
    for q in range(4):
        assert rel_rms(got[q], ind[q]) < tol, q
        assert abs(gsw[q] - sws[q]) <= 1e-12 * abs(sws[q])
    if path == "fused":
        assert info["nvis_used"] == nrow * nchan  # (every in-grid visibility bucketed)


@pytest.mark.parametrize("path", ["fine", "coarse", "fp64"])
@pytest.mark.parametrize("vdt", [torch.complex64, torch.complex128])
@pytest.mark.parametrize("acc", [False, True])
def test_predict_pols_call_matches_per_pol_calls(path, vdt, acc, monkeypatch):
    """sdp_hip_dirty2ms_vis_pols (predict_ng's image pols in one call: one
    bucketing, each pol's planes and degridding, one write-back through the
    conversion matrix) against one dirty2ms_vis call per image pol (the first
    without, the others with accumulation): stokesIQUV -> linear, with and
    without accumulation into the output; 16x16-cell buckets ("coarse") and
    the fp64 path (epsilon 1e-12) too.  1e-6 relative RMS (fp32 sums of the
    pols in the output dtype vs one fp64 sum)."""
    from ska_sdp_func_python_amd import kernels
    if path == "coarse":
        monkeypatch.setenv("SDP_HIP_BUCKET", "16")
    rng = np.random.default_rng(73)
    nrow, nchan, npv, npix = 4000, 5, 4, 128
    freq = np.linspace(1.0e9, 1.2e9, nchan)
    umax = 3000.0
    uvw_h = rng.uniform(-1, 1, (nrow, 3)) * umax * orc.C_LIGHT / freq.max()
    uvw_h[:, 2] *= 0.3
    dev = "cuda"
    uvw = torch.as_tensor(uvw_h, device=dev)
    freq_t = torch.as_tensor(freq, device=dev)
    imgs = torch.as_tensor(rng.normal(size=(4, npix, npix)), device=dev)
    # IQUV -> linear: column q of the conversion = image pol q's vis pols
    cols = [[1, 0, 0, 1], [1, 0, 0, -1], [0, 1, 1, 0], [0, 1j, -1j, 0]]
    cell = 0.35 / umax
    eps = 1e-12 if path == "fp64" else 1e-5
    base = torch.as_tensor(rng.normal(size=(nrow, nchan, npv)) +
                           1j * rng.normal(size=(nrow, nchan, npv)), device=dev).to(vdt)
    ref = base.clone() if acc else torch.zeros_like(base)
    for q in range(4):
        kernels.dirty2ms_vis(uvw, freq_t, imgs[q], ref, cols[q], cell, cell, eps, True,
                             flip_uw=True, accumulate=acc or q > 0)
    got = base.clone() if acc else torch.full_like(base, float("nan"))
    kernels.dirty2ms_vis_pols(uvw, freq_t, imgs, got, cols, cell, cell, eps, True, flip_uw=True,
                              accumulate=acc)
    tol = 1e-12 if (path == "fp64" and vdt == torch.complex128) else 1e-6
    assert rel_rms(got.cpu().numpy(), ref.cpu().numpy()) < tol


@pytest.mark.parametrize("ipf,pf", [("stokesI", "stokesI"), ("stokesIQUV", "linear"),
                                    ("stokesIQUV", "circular"), ("linear", "linear")])
@pytest.mark.parametrize("mfs", [True, False])
@pytest.mark.parametrize("device", [False, True])
def test_predict_ng_fused_pol_conversion(ipf, pf, mfs, device):
    """predict_ng writes each image pol's prediction times its column of the
    conversion matrix (ng.py:131-136) straight into the output Visibility
    (sdp_hip_dirty2ms_vis), in the input's dtype; against exact sums + numpy
    conversion, TOL relative RMS per vis pol."""
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.imaging import predict_ng
    rng = np.random.default_rng(23)
    nt, nb, nchan = 4, 30, 3
    npol = dm.PolarisationFrame(pf).npol
    freq = np.linspace(1.0e9, 1.1e9, nchan)
    umax = 1500.0
    uvw = rng.uniform(-1, 1, (nt, nb, 3)) * umax * orc.C_LIGHT / freq.max()
    uvw[..., 2] *= 0.5
    shape = (nt, nb, nchan, npol)
    vis = vis_from_arrays(uvw, freq, np.zeros(shape, complex), pf=pf,
                          phasecentre=dm.SkyCoord(0.0, -0.6))
    npix, cell = 96, 0.4 / umax
    fc, bw = (float(freq.mean()), 1e9) if mfs else (float(freq[0]), float(freq[1] - freq[0]))
    im = dm.create_image(npix, cell, dm.SkyCoord(0.0, -0.6), polarisation_frame=dm.PolarisationFrame(ipf),
                         frequency=fc, channel_bandwidth=bw, nchan=1 if mfs else nchan)
    im["pixels"].data[...] = rng.normal(size=im["pixels"].data.shape)
    fuvw = uvw.reshape(-1, 3) * FLIP_UW
    nimch = 1 if mfs else nchan
    pred = np.zeros((nt * nb, nchan, npol), complex)
    for p in range(npol):
        for c in range(nchan):
            ic = 0 if mfs else c
            pred[:, c, p] = orc.dirty2ms_exact(fuvw, freq[c:c + 1], im["pixels"].data[ic, p].T, None,
                                               cell, cell, True)[:, 0]
    expect = dm.convert_pol_frame(pred, im.image_acc.polarisation_frame,
                                  vis.visibility_acc.polarisation_frame, polaxis=2)
    if device:
        vis["vis"] = torch.zeros(shape, dtype=torch.complex64, device="cuda")
        vis["uvw"] = torch.as_tensor(uvw, device="cuda")
    out = predict_ng(vis, im)
    got = out.vis.data
    if device:
        assert got.dtype == torch.complex64
        got = got.cpu().numpy()
    else:
        assert got.dtype == np.complex128
    got = got.reshape(nt * nb, nchan, npol)
    for p in range(npol):
        assert rel_rms(got[..., p], expect[..., p]) < TOL, p
    assert nimch in (1, nchan)


@pytest.mark.parametrize("device", [False, True])
def test_fused_phase_shift_invert_and_predict(device):
    """An image whose phase centre is offset from the visibilities' (0.01 rad
    in RA, 0.007 in Dec): shift_vis_to_image's tangent-plane rotation
    (imaging/base.py:48-92, visibility/base.py:27-90) is applied inside the
    fused kernels; against the numpy rotation + exact sums (TOL), and the
    returned predict Visibility is relabelled to the image phase centre."""
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.imaging import invert_ng, predict_ng
    from ska_sdp_func_python_amd.util.coordinate_support import skycoord_to_lmn
    rng = np.random.default_rng(29)
    nt, nb, nchan = 5, 40, 2
    freq = np.linspace(1.0e9, 1.1e9, nchan)
    umax = 1500.0
    uvw = rng.uniform(-1, 1, (nt, nb, 3)) * umax * orc.C_LIGHT / freq.max()
    uvw[..., 2] *= 0.5
    shape = (nt, nb, nchan, 1)
    v = rng.normal(size=shape) + 1j * rng.normal(size=shape)
    vpc = dm.SkyCoord(0.3, -0.6)
    ipc = dm.SkyCoord(0.31, -0.593)
    vis = vis_from_arrays(uvw, freq, v, phasecentre=vpc)
    npix, cell = 128, 0.4 / umax
    im = dm.create_image(npix, cell, ipc, frequency=float(freq.mean()), channel_bandwidth=1e9)
    l, m, n = skycoord_to_lmn(dm.pixel_to_skycoord(npix // 2 + 1, npix // 2 + 1, im.image_acc.wcs,
                                                   origin=1), vpc)
    assert abs(n) > 1e-6
    d = np.einsum("tbs,s->tb", uvw, [l, m, n])[..., None] * freq / orc.C_LIGHT  # turns [t,b,f]
    fuvw = uvw.reshape(-1, 3) * FLIP_UW
    rot = v[..., 0] * np.exp(2j * np.pi * d)
    ref = orc.ms2dirty_exact(fuvw, freq, rot.reshape(-1, nchan), None, npix, npix, cell, cell,
                             True).T / (nt * nb * nchan)
    model = im.copy(deep=True)
    model["pixels"].data[0, 0] = rng.normal(size=(npix, npix))
    pred = orc.dirty2ms_exact(fuvw, freq, model["pixels"].data[0, 0].T, None, cell, cell, True)
    pred = pred.reshape(nt, nb, nchan) * np.exp(-2j * np.pi * d)
    if device:
        vis["vis"] = torch.as_tensor(v, device="cuda")
        vis["uvw"] = torch.as_tensor(uvw, device="cuda")
    dirty, _ = invert_ng(vis, im)
    img = dirty["pixels"].data
    img = img.cpu().numpy() if device else img
    assert rel_rms(img[0, 0], ref) < TOL
    out = predict_ng(vis, model)
    got = out.vis.data.cpu().numpy() if device else out.vis.data
    assert rel_rms(got[..., 0], pred) < TOL
    assert out.phasecentre.separation(ipc).rad < 1e-12


@pytest.mark.parametrize("flip", [False, True])
def test_batched_invert_equals_single_call(flip, monkeypatch):
    """sdp_hip_ms2dirty_batch: three channel blocks gridded into shared
    resident planes and transformed once equal one ms2dirty over all the
    channels (same plane layout from the merged bounds); a plane layout that
    does not fit the device is refused."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(21, nrow=4000, nchan=6, umax=6000.0)
    U, F, M, Wt = T(uvw), T(freq), T(ms), T(wgt)
    full, info = kernels.ms2dirty(U, F, M, Wt, 256, 192, cell, cell, 1e-7, True, flip_uw=flip)
    blocks = [(0, 2), (2, 3), (3, 6)]
    b = kernels.merge_bounds(*[kernels.uvw_bounds(U, F[a:e]) for a, e in blocks])
    out = None
    for i, (a, e) in enumerate(blocks):
        out, binfo = kernels.ms2dirty_batch(U, F[a:e], M[:, a:e].contiguous(),
                                            Wt[:, a:e].contiguous(), 256, 192, cell, cell, b,
                                            first=i == 0, last=i == len(blocks) - 1,
                                            epsilon=1e-7, flip_uw=flip)
        assert (out is None) == (i < len(blocks) - 1)
        assert binfo["nplanes"] == info["nplanes"] and binfo["w0"] == info["w0"]
    assert rel_rms(out.cpu().numpy(), full.cpu().numpy()) < 1e-6
    exact = orc.ms2dirty_exact(uvw * (FLIP_UW if flip else 1.0), freq, ms, wgt, 256, 192, cell,
                               cell, True)
    assert rel_rms(out.cpu().numpy(), exact) < TOL
    monkeypatch.setenv("SDP_HIP_GRID_BUDGET_GB", "0.0001")
    with pytest.raises(ValueError, match="do not all fit"):
        kernels.ms2dirty_batch(U, F[:2], M[:, :2].contiguous(), None, 256, 192, cell, cell, b,
                               first=True, last=False, epsilon=1e-7)


def test_batch_bounds_too_tight_are_refused():
    """A batch of a batched invert whose visibilities fall outside the
    sequence's bounds (u beyond max|u|, or w beyond the w range) is refused
    with ValueError instead of indexing outside the histogram / planes."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(22, nrow=2000, nchan=3, umax=6000.0)
    uvw[:, 2] *= 200.0  # w spans many planes at this field of view
    U, F, M = T(uvw), T(freq), T(ms)
    b = kernels.uvw_bounds(U, F)
    for tight in ([b[0], b[1], 0.5 * b[2], b[3], b[4], b[5]],           # u range too small
                  [b[0], 0.5 * (b[0] + b[1]), b[2], b[3], b[4], b[5]],   # w range too small
                  [b[0], b[1], b[2], b[3], 0.7 * b[4], 0.7 * b[5]]):     # frequencies too low
        with pytest.raises(ValueError, match="outside"):
            kernels.ms2dirty_batch(U, F, M, None, 256, 256, cell, cell, tight, first=True,
                                   last=True, epsilon=1e-7)
    out, _ = kernels.ms2dirty_batch(U, F, M, None, 256, 256, cell, cell, b, first=True,
                                    last=True, epsilon=1e-7)
    ref, _ = kernels.ms2dirty(U, F, M, None, 256, 256, cell, cell, 1e-7, True)
    assert rel_rms(out.cpu().numpy(), ref.cpu().numpy()) < 1e-6


def test_batch_sequence_guard():
    """The resident planes of a batch sequence belong to it until its last
    batch: another NUFFT call or a workspace release in between, or a batch
    with other bounds / geometry, makes the next batch fail with ValueError
    rather than accumulate into overwritten or freed planes."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, _, cell = _problem(23, nrow=2000, nchan=4, umax=5000.0)
    U, F, M = T(uvw), T(freq), T(ms)
    b = kernels.merge_bounds(kernels.uvw_bounds(U, F[:2]), kernels.uvw_bounds(U, F[2:]))
    args = (256, 256, cell, cell)

    def batch(i, bb=b, first=False, last=False, npix=256):
        return kernels.ms2dirty_batch(U, F[2 * i:2 * i + 2], M[:, 2 * i:2 * i + 2].contiguous(),
                                      None, npix, npix, cell, cell, bb, first=first, last=last,
                                      epsilon=1e-7)

    batch(0, first=True)
    kernels.ms2dirty(U, F, M, None, *args, 1e-7, True)  # another call overwrites the planes
    with pytest.raises(ValueError, match="no resident planes"):
        batch(1, last=True)
    batch(0, first=True)
    kernels.release_workspace()
    with pytest.raises(ValueError, match="no resident planes"):
        batch(1, last=True)
    batch(0, first=True)
    wider = list(b)
    wider[2] *= 1.01
    with pytest.raises(ValueError, match="first batch|no resident planes"):
        batch(1, bb=wider, last=True)
    # an uninterrupted sequence still equals the single call
    batch(0, first=True)
    out, _ = batch(1, last=True)
    ref, _ = kernels.ms2dirty(U, F, M, None, *args, 1e-7, True)
    assert rel_rms(out.cpu().numpy(), ref.cpu().numpy()) < 1e-6
    with pytest.raises(ValueError, match="no resident planes"):  # the sequence has ended
        batch(1, last=True)


def test_f64_weights_in_the_bare_entries():
    """ducc0's ms2dirty / dirty2ms take f64 weights: the bare C ABI entries
    accept f64 (and f32) weights, with identical results for weights exact in
    both precisions, and match the exact sums."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(24)
    w64 = np.round(wgt.astype(np.float64) * 64) / 64
    ex = orc.ms2dirty_exact(uvw, freq, ms, w64, 64, 64, cell, cell, True)
    a, _ = kernels.ms2dirty(T(uvw), T(freq), T(ms), T(w64), 64, 64, cell, cell, 1e-7, True)
    b, _ = kernels.ms2dirty(T(uvw), T(freq), T(ms), T(w64, torch.float32), 64, 64, cell, cell,
                            1e-7, True)
    # (the flush atomics make the fp32 sum order vary from run to run)
    assert rel_rms(a.cpu().numpy(), b.cpu().numpy()) < 1e-6
    assert rel_rms(a.cpu().numpy(), ex) < TOL
    img = np.random.default_rng(3).normal(size=(64, 64))
    vx = orc.dirty2ms_exact(uvw, freq, img, w64, cell, cell, True)
    v, _ = kernels.dirty2ms(T(uvw), T(freq), T(img), T(w64), cell, cell, 1e-7, True)
    assert rel_rms(v.cpu().numpy(), vx) < TOL


@pytest.mark.parametrize("pf,ipf", [("linear", "stokesIQUV"), ("stokesI", "stokesI")])
def test_nan_in_flagged_samples_does_not_reach_the_image(pf, ipf):
    """NaN / Inf visibilities and weights on flagged samples, and NaN / Inf
    visibilities on samples whose weights are zero in every pol, contribute
    nothing, as ducc0 skips zero-weight samples: invert_ng (multi-pol: shared
    bucketing across the image pols, which buckets zero-weight samples too)
    equals the same call with those values replaced by zeros.  (An unflagged
    non-finite visibility of a pol with zero weight still enters the other
    image pols through the pol conversion, as it does in the reference's
    numpy convert_pol_frame -- not exercised here.)"""
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.imaging import invert_ng
    rng = np.random.default_rng(31)
    nt, nb, nchan = 4, 40, 3
    npol = dm.PolarisationFrame(pf).npol
    freq = np.linspace(1.0e9, 1.1e9, nchan)
    umax = 1500.0
    uvw = rng.uniform(-1, 1, (nt, nb, 3)) * umax * orc.C_LIGHT / freq.max()
    shape = (nt, nb, nchan, npol)
    v = rng.normal(size=shape) + 1j * rng.normal(size=shape)
    w = rng.uniform(0.5, 2.0, shape)
    fl = (rng.uniform(size=shape) < 0.2).astype(int)
    zw = np.broadcast_to(rng.uniform(size=shape[:3] + (1,)) < 0.1, shape)
    w[zw] = 0.0
    bad_v, bad_w = v.copy(), w.copy()
    bad_v[fl == 1] = np.nan
    bad_v[zw] = complex(np.inf, np.nan)
    bad_w[fl == 1] = np.nan
    im = dm.create_image(96, 0.4 / umax, dm.SkyCoord(0.0, -0.6),
                         polarisation_frame=dm.PolarisationFrame(ipf), frequency=float(freq.mean()),
                         channel_bandwidth=1e9)
    clean_v = np.where(fl == 1, 0.0, v)
    clean_v[zw] = 0.0
    res = []
    for vv, ww in ((bad_v, bad_w), (clean_v, np.where(fl == 1, 0.0, w))):
        vis = vis_from_arrays(uvw, freq, vv, flags=fl, pf=pf, phasecentre=dm.SkyCoord(0.0, -0.6))
        vis["imaging_weight"] = ww
        res.append(invert_ng(vis, im, normalise=False))
    (d_bad, sw_bad), (d_ok, sw_ok) = res
    assert np.all(np.isfinite(d_bad["pixels"].data)) and np.all(np.isfinite(sw_bad))
    np.testing.assert_allclose(sw_bad, sw_ok, rtol=1e-12)
    for p in range(npol):
        assert rel_rms(d_bad["pixels"].data[0, p], d_ok["pixels"].data[0, p]) < 1e-6, p


@pytest.mark.parametrize("flip", [False, True])
def test_w_slabs_sum_to_the_full_invert(flip):
    """SDP_HIP_W_SLAB (the multi-GPU w-slab partition): the dirty images of
    contiguous first-plane slabs of one plane layout -- each a batched
    sequence over the whole band that grids only its slab's visibilities into
    its slab's planes -- sum to the full invert; the slabs' gridded
    visibilities add up to the total and each holds only its slab's planes
    (+ W - 1); visibilities outside the layout are still refused."""
    from ska_sdp_func_python_amd import kernels, parallel
    uvw, freq, ms, wgt, cell = _problem(24, nrow=3000, nchan=6, umax=6000.0)
    uvw[:, 2] *= 60.0  # w spans many planes
    U, F, M, Wt = T(uvw), T(freq), T(ms), T(wgt)
    blocks = [(0, 2), (2, 4), (4, 6)]
    b = kernels.merge_bounds(*[kernels.uvw_bounds(U, F[a:e]) for a, e in blocks])
    full = None
    for i, (a, e) in enumerate(blocks):
        full, finfo = kernels.ms2dirty_batch(U, F[a:e], M[:, a:e].contiguous(),
                                             Wt[:, a:e].contiguous(), 256, 256, cell, cell, b,
                                             first=i == 0, last=i == 2, epsilon=1e-7,
                                             flip_uw=flip)
    lay = kernels.wstack_layout(b, 256, 256, cell, cell, 1e-7, True, flip_uw=flip)
    assert lay["nplanes"] == finfo["nplanes"] and lay["w0"] == finfo["w0"]
    nps, W = lay["nps"], lay["support"]
    assert nps >= 6
    hist = parallel.first_plane_histogram(U, freq, lay, flip_uw=flip)
    assert hist.sum() == uvw.shape[0] * freq.size
    slabs = parallel.wslab_partition(hist, 3, W)
    assert slabs[0][0] == 0 and slabs[-1][1] == nps
    assert all(s[1] == t[0] for s, t in zip(slabs, slabs[1:]))
    total = torch.zeros_like(full)
    used = 0
    for lo, hi in slabs + [(nps, nps + 5)]:  # (a slab past the layout grids nothing)
        if lo >= hi or lo >= nps:
            continue
        out = None
        for i, (a, e) in enumerate(blocks):
            out, sinfo = kernels.ms2dirty_batch(U, F[a:e], M[:, a:e].contiguous(),
                                                Wt[:, a:e].contiguous(), 256, 256, cell, cell, b,
                                                first=i == 0, last=i == 2, epsilon=1e-7,
                                                flip_uw=flip, slab=(lo, hi))
            used += sinfo["nvis_used"]
        assert sinfo["nplanes"] == min(hi, nps) - lo + W - 1
        assert abs(sinfo["w0"] - (lay["w0"] + lo * lay["dw"])) < 1e-9 * abs(lay["dw"]) * nps
        total += out
    assert used == uvw.shape[0] * freq.size
    assert rel_rms(total.cpu().numpy(), full.cpu().numpy()) < 1e-6
    exact = orc.ms2dirty_exact(uvw * (FLIP_UW if flip else 1.0), freq, ms, wgt, 256, 256, cell,
                               cell, True)
    assert rel_rms(total.cpu().numpy(), exact) < TOL
    tight = [b[0], 0.5 * (b[0] + b[1]), b[2], b[3], b[4], b[5]]
    with pytest.raises(ValueError, match="outside"):
        kernels.ms2dirty_batch(U, F, M, None, 256, 256, cell, cell, tight, first=True, last=True,
                               epsilon=1e-7, flip_uw=flip, slab=(0, 1))


def test_row_partition_by_w_sums_to_the_full_invert():
    """parallel.wrow_partition (the C4 strong-scaling partition): rows cut
    into contiguous w intervals, each inverted over all channels with its OWN
    w-plane layout (fewer planes for the small-|w| intervals); the images sum
    to the full invert and to the exact sums."""
    from ska_sdp_func_python_amd import kernels, parallel
    uvw, freq, ms, wgt, cell = _problem(25, nrow=4000, nchan=5, umax=6000.0)
    uvw[:, 2] *= 60.0
    U, F, M, Wt = T(uvw), T(freq), T(ms), T(wgt)
    full, info = kernels.ms2dirty(U, F, M, Wt, 256, 256, cell, cell, 1e-7, True, flip_uw=True)
    order, cuts, costs = parallel.wrow_partition(-uvw[:, 2], freq, 3, info["dw"], info["support"])
    assert cuts[0] == 0 and cuts[-1] == uvw.shape[0] and len(costs) == 3
    total = torch.zeros_like(full)
    planes = []
    for r in range(3):
        rows = torch.as_tensor(order[cuts[r]:cuts[r + 1]], device="cuda")
        part, pinfo = kernels.ms2dirty(U[rows].contiguous(), F, M[rows].contiguous(),
                                       Wt[rows].contiguous(), 256, 256, cell, cell, 1e-7, True,
                                       flip_uw=True)
        planes.append(pinfo["nplanes"])
        total += part
    assert min(planes) < info["nplanes"]
    assert rel_rms(total.cpu().numpy(), full.cpu().numpy()) < 1e-6
    exact = orc.ms2dirty_exact(uvw * FLIP_UW, freq, ms, wgt, 256, 256, cell, cell, True)
    assert rel_rms(total.cpu().numpy(), exact) < TOL


def test_two_slots_on_two_streams_overlap_correctly():
    """SDP_HIP_SLOT1: inverts alternated between two streams and the library's
    two scratch slots (the pipelined bench) -- different problems in flight at
    once -- each equal to its own single call; slot 1 refuses batches."""
    from ska_sdp_func_python_amd import kernels
    probs = [_problem(30 + k, nrow=3000, nchan=4, umax=5000.0) for k in range(2)]
    dev = torch.device("cuda:0")
    refs = []
    for uvw, freq, ms, wgt, cell in probs:
        r, _ = kernels.ms2dirty(T(uvw), T(freq), T(ms), T(wgt), 256, 256, cell, cell, 1e-7, True)
        refs.append(r.cpu().numpy())
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    args = [(T(uvw), T(freq), T(ms), T(wgt), cell) for uvw, freq, ms, wgt, cell in probs]
    torch.cuda.synchronize()
    outs = [[], []]
    for rep in range(3):
        for j in (0, 1):
            U, F, M, Wt, cell = args[j]
            with torch.cuda.stream(streams[j]):
                o, _ = kernels.ms2dirty(U, F, M, Wt, 256, 256, cell, cell, 1e-7, True, slot=j)
            outs[j].append(o)
    torch.cuda.synchronize()
    for j in (0, 1):
        for o in outs[j]:
            assert rel_rms(o.cpu().numpy(), refs[j]) < 1e-6
    U, F, M, Wt, cell = args[0]
    b = kernels.uvw_bounds(U, F)
    import ctypes
    with pytest.raises(ValueError, match="SLOT1"):
        bbuf = (ctypes.c_double * 6)(*b)
        info = kernels._lib.WGridInfo()
        kernels._lib.call("sdp_hip_ms2dirty_batch", kernels._ptr(U), U.stride(0), kernels._ptr(F),
                          F.shape[0], U.shape[0], kernels._ptr(M), kernels._lib.SDP_HIP_C64,
                          M.stride(0), M.stride(1), None, kernels._lib.SDP_HIP_F32, 0, 0, 256, 256,
                          cell, cell, 1e-7, 1,
                          kernels._lib.SDP_HIP_SLOT1 | kernels._lib.SDP_HIP_BATCH_FIRST,
                          ctypes.cast(bbuf, ctypes.c_void_p), None, 0, 0,
                          kernels._stream(dev), ctypes.byref(info))


def test_invert_after_workspace_release_is_unchanged():
    """The band-only x-FFT input keeps its zeros across calls: after
    release_workspace a new allocation (possibly at the same address, holding
    stale data) must be cleared again (band state keyed by the allocation's
    workspace epoch, not its address)."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(21, nrow=2000, nchan=4, umax=4000.0)
    args = (T(uvw), T(freq), T(ms), T(wgt), 256, 256, cell, cell, 1e-7, True)
    a, _ = kernels.ms2dirty(*args)
    kernels.release_workspace()
    # dirty the freed memory so that a re-allocation at the same address sees garbage
    junk = torch.full((64 << 20,), float("nan"), device=dev())
    del junk
    torch.cuda.empty_cache()
    b, _ = kernels.ms2dirty(*args)
    assert torch.isfinite(b).all()
    assert rel_rms(b.cpu().numpy(), a.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("npix,ny,dow", [(64, 48, True), (128, 128, False), (256, 200, True),
                                         (1024, 1024, True), (2048, 1536, True),
                                         (4096, 4096, True), (8192, 256, True)])
def test_fused_xfft_screens_match_hipfft(npix, ny, dow, monkeypatch):
    """The fused x-FFT + screen kernels (k_xfft_screen_fwd / k_screen_adj_xfft,
    ngx = 2^7 .. 2^14) against hipFFT + the separate screens
    (SDP_HIP_XFFT_FUSED=0), invert and predict: both are fp32 transforms of
    the same planes, so they agree to fp32 rounding."""
    from ska_sdp_func_python_amd import kernels
    uvw, freq, ms, wgt, cell = _problem(11, nrow=4000, nchan=4, umax=2e4 * npix / 4096)
    rng = np.random.default_rng(12)
    img = rng.normal(size=(npix, ny))
    outs = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("SDP_HIP_XFFT_FUSED", fused)
        d, _ = kernels.ms2dirty(T(uvw), T(freq), T(ms), T(wgt), npix, ny, cell, cell * 0.9, 1e-7,
                                dow, flip_uw=True)
        v, _ = kernels.dirty2ms(T(uvw), T(freq), T(img), T(wgt), cell, cell * 0.9, 1e-7, dow,
                                flip_uw=True)
        outs[fused] = (d.cpu().numpy(), v.cpu().numpy())
    assert rel_rms(outs["1"][0], outs["0"][0]) < 1e-6
    assert rel_rms(outs["1"][1], outs["0"][1]) < 1e-6
