"""Parity of the HIP w-stacking NUFFT on the FULL headline workload (C2:
SKA-MID 197 dishes x 100 times x 64 channels = 123.6 Mvis, 4096^2 image on the
8192^2 w-stacked grid -- bench.py's step) against the reference-precision
oracle:

* oracle/wgrid_cpu.c with precision="double": epsilon 1e-12 -> W = 13, fp64
  taps, fp64 planes, i.e. the reference's ducc0 call
  (src/ska_sdp_func_python/imaging/ng.py:240-256, double_precision_accumulation
  =True; ducc0 itself is absent, "parity unpinned" at that boundary);
* the exact direct sums ducc0 approximates, at sampled pixels / rows, as the
  absolute anchor of both.

Tolerance (north star): dirty-image / visibility RMS error < 1e-5 relative to
the RMS of the reference-precision result.  Measured values are printed
(`pytest -s`) and recorded in DESIGN.md §5.
"""

import math

import numpy as np
import pytest
import torch

from conftest import rel_rms

pytestmark = pytest.mark.gpu
TOL = 1e-5
FLIP_UW = np.array([-1.0, 1.0, -1.0])
NPIX = 4096
F_LO, F_HI = 0.95e9, 1.76e9


def _c2():
    from ska_sdp_func_python_amd import simulation
    dev = torch.device("cuda:0")
    obs = simulation.device_observation(100, 64, F_LO, F_HI, config="MID", seed=0, device=dev)
    return obs, 0.25 / obs["umax"]


@pytest.fixture(autouse=True)
def _free_device_memory():
    """Full-size cases hold up to ~250 GB of HBM (C4 shard: 150 GB of resident
    w planes in the library's cached workspace); release it between tests."""
    yield
    import gc
    from ska_sdp_func_python_amd import kernels
    gc.collect()
    torch.cuda.synchronize()
    kernels.release_workspace()
    torch.cuda.empty_cache()


def _threads():
    import os
    return min(16, len(os.sched_getaffinity(0)))


@pytest.mark.timeout(900)
def test_c2_full_invert_against_reference_precision():
    import wgrid_cpu
    from ska_sdp_func_python_amd import kernels
    obs, cell = _c2()
    assert obs["nrow"] * 64 == 123_558_400
    out, info = kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], NPIX, NPIX,
                                 cell, cell, 1e-7, True, flip_uw=True)
    gpu = out.cpu().numpy()
    # the reference's default precision on the GPU: epsilon 1e-12, the fp64
    # NUFFT (W = 13, the same algorithm as the oracle) -- equal to 1e-10
    out, info64 = kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], NPIX, NPIX,
                                   cell, cell, 1e-12, True, flip_uw=True)
    assert info64["fp64"] == 1 and info64["support"] == 13
    gpu64 = out.cpu().numpy()
    uvw = obs["uvw"].cpu().numpy() * FLIP_UW
    freq = obs["freq"].cpu().numpy()
    ms = obs["vis"].cpu().numpy()
    wgt = obs["wgt"].cpu().numpy()
    del out, obs
    torch.cuda.empty_cache()
    oinfo = {}
    ref, tg, tf = wgrid_cpu.ms2dirty(uvw, freq, ms, wgt, NPIX, NPIX, cell, cell, 1e-12, True,
                                     nthreads=_threads(), precision="double", info=oinfo)
    assert oinfo["support"] == 13
    err = rel_rms(gpu, ref)
    # absolute anchor: exact direct sums at 48 pixels (centre, axes, corners, random)
    rng = np.random.default_rng(31)
    px = np.concatenate([[NPIX // 2, NPIX // 2, 0, NPIX - 1, NPIX // 2 + 1],
                         rng.integers(0, NPIX, 43)])
    py = np.concatenate([[NPIX // 2, 0, NPIX // 2, NPIX - 1, NPIX // 2 - 7],
                         rng.integers(0, NPIX, 43)])
    ex = wgrid_cpu.exact_pixels(uvw, freq, ms, wgt, NPIX, NPIX, cell, cell, True, px, py,
                                nthreads=_threads())
    e_ref = rel_rms(ref[px, py], ex)
    e_gpu = rel_rms(gpu[px, py], ex)
    err64 = rel_rms(gpu64, ref)
    e_gpu64 = rel_rms(gpu64[px, py], ex)
    print(f"\nC2 full invert (123.6 Mvis, W_gpu={info['support']}, planes={info['nplanes']}): "
          f"rel-RMS GPU vs fp64 W=13 oracle {err:.3e}; at 48 exact pixels: GPU {e_gpu:.3e}, "
          f"oracle {e_ref:.3e} (oracle grid {tg:.1f} s, fft {tf:.1f} s); GPU fp64 (epsilon "
          f"1e-12, {info64['nplanes']} planes) vs oracle {err64:.3e}, at the exact pixels "
          f"{e_gpu64:.3e}")
    assert e_ref < 1e-9
    assert e_gpu < TOL
    assert err < TOL
    assert err64 < 1e-10 and e_gpu64 < 1e-9


@pytest.mark.timeout(900)
def test_c2_full_predict_against_reference_precision():
    import wgrid_cpu
    from ska_sdp_func_python_amd import kernels
    obs, cell = _c2()
    rng = np.random.default_rng(32)
    img = rng.normal(size=(NPIX, NPIX))
    v, info = kernels.dirty2ms(obs["uvw"], obs["freq"], torch.as_tensor(img, device="cuda:0"),
                               obs["wgt"], cell, cell, 1e-7, True, flip_uw=True)
    gpu = v.cpu().numpy()
    del v
    v, _ = kernels.dirty2ms(obs["uvw"], obs["freq"], torch.as_tensor(img, device="cuda:0"),
                            obs["wgt"], cell, cell, 1e-12, True, flip_uw=True,
                            vis_dtype=torch.complex128)
    gpu64 = v.cpu().numpy()
    uvw = obs["uvw"].cpu().numpy() * FLIP_UW
    freq = obs["freq"].cpu().numpy()
    wgt = obs["wgt"].cpu().numpy()
    nrow = obs["nrow"]
    del v, obs
    torch.cuda.empty_cache()
    ref, tg, tf = wgrid_cpu.dirty2ms(uvw, freq, img, wgt, cell, cell, 1e-12, True,
                                     nthreads=_threads(), precision="double")
    err = rel_rms(gpu, ref)
    rows = np.sort(rng.choice(nrow, 24, replace=False))
    ex = wgrid_cpu.exact_rows(uvw, freq, img, rows, cell, cell, True, nthreads=_threads())
    e_ref = rel_rms(ref[rows], ex)
    e_gpu = rel_rms(gpu[rows], ex)
    err64 = rel_rms(gpu64, ref)
    print(f"\nC2 full predict (123.6 Mvis, W_gpu={info['support']}): rel-RMS GPU vs fp64 W=13 "
          f"oracle {err:.3e}; 24 exact rows x 64 chans: GPU {e_gpu:.3e}, oracle {e_ref:.3e} "
          f"(oracle degrid {tg:.1f} s, fft {tf:.1f} s); GPU fp64 vs oracle {err64:.3e}")
    assert e_ref < 1e-9
    assert e_gpu < TOL
    assert err < TOL
    assert err64 < 1e-10


# ---------------------------------------------------------------------------
# C3: dft_skycomponent_visibility, 1000 point components x 10 Mvis
# ---------------------------------------------------------------------------
@pytest.mark.timeout(600)
@pytest.mark.parametrize("vdt", [torch.complex64, torch.complex128])
def test_c3_dft_full_against_fp64_reference(vdt):
    """C3 (SKA-MID 197 dishes x 518 times x 1 channel = 10.0 Mvis, 1000
    components, l, m in +-0.05 rad, flux U(0.1, 10) Jy): 4096 sampled
    visibilities against the reference's dft_cpu_looped restated in fp64
    (oracle/ref_oracle.py, pinned to the reference-run dft fixtures).  The
    phase is fp64 reduced to turns, sin/cos fp32 (revolutions): relative
    RMS < 2e-6 for both outputs; complex128 output accumulates in fp64."""
    import ref_oracle as ro
    from ska_sdp_func_python_amd import kernels, simulation
    fn, n_def, lat, dec = simulation.CONFIGS["MID"]
    ha = np.linspace(-0.5, 0.5, 518) * 8.0 * math.pi / 12.0
    uvw_h, _ = simulation.observe(fn(n_def, seed=1), math.radians(lat), math.radians(dec), ha)
    uvw_h = uvw_h.reshape(-1, 3)
    assert uvw_h.shape[0] == 10_000_508
    rng = np.random.default_rng(3)
    lm = rng.uniform(-0.05, 0.05, (1000, 2))
    dc = np.concatenate([lm, (np.sqrt(1 - (lm ** 2).sum(1)) - 1)[:, None]], 1)
    flux = rng.uniform(0.1, 10, (1000, 1, 1)).astype(complex)
    freq = np.array([1.4e9])
    dev = torch.device("cuda:0")
    out = kernels.dft_point(torch.as_tensor(dc, device=dev), torch.as_tensor(flux, device=dev),
                            torch.as_tensor(uvw_h, device=dev),
                            freq=torch.as_tensor(freq, device=dev), vis_dtype=vdt)
    rows = np.sort(rng.choice(uvw_h.shape[0], 4096, replace=False))
    got = out[torch.as_tensor(rows, device=dev)].cpu().numpy()
    uvwl = uvw_h[rows][:, None, :] * (freq / 299792458.0)[None, :, None]
    ref = ro.dft_cpu_looped(dc, uvwl[None], flux)[0]
    err = rel_rms(got, ref)
    print(f"\nC3 DFT (10.0 Mvis x 1000 comps, {vdt}): rel-RMS vs fp64 dft_cpu_looped {err:.2e}")
    assert err < 2e-6


# ---------------------------------------------------------------------------
# C4: one rank's shard of the SKA-LOW 8192^2 invert (1.67 Gvis, 16384^2 grid)
# ---------------------------------------------------------------------------
@pytest.mark.timeout(1200)
def test_c4_shard_invert_predict_at_full_size():
    """SKA-LOW 512 stations x 400 times x 32 of the 256 channels (the top
    block of the band, 1.67 Gvis, the most w planes of any rank) on the
    8192^2 image / 16384^2 grid: adjointness <A x, y> = Re <x, A^H y> over
    all 1.67 Gvis, a unit point source predicts |V| = 1/n exactly and its
    dirty image peaks at the source with the value sum(w)/n^2, and the dirty
    image of the random visibilities against exact direct sums at sampled
    pixels (oracle/wgrid_cpu.c).

    The benchmarked C4 path, sdp_hip_ms2dirty_batch, runs the same shard as 3
    channel batches sharing the top band's plane layout (> 40 resident 16384^2
    planes): equal to the single call (5e-6: fp32 sums in another order) and
    to the exact pixels.

    Device-memory policy: the whole sequence runs in one process with no
    workspace release -- a smaller 16384^2 invert first (its planes cached),
    then the shard's invert (150 GB of planes), predicts whose outputs
    (12.5 GiB) torch allocates beside the cached planes, the batched
    inverts, and finally a 16 GiB torch allocation."""
    import wgrid_cpu
    from ska_sdp_func_python_amd import kernels, simulation
    dev = torch.device("cuda:0")
    npix = 8192
    # a 16384^2 invert of another problem first: its planes stay cached
    rs = np.random.default_rng(40)
    u_s = rs.uniform(-1, 1, (20000, 3)) * 3.0e5 * 299792458.0 / 1.2e9
    u_s[:, 2] *= 0.02
    f_s = np.linspace(1.0e9, 1.2e9, 4)
    m_s = rs.normal(size=(20000, 4)) + 1j * rs.normal(size=(20000, 4))
    kernels.ms2dirty(torch.as_tensor(u_s, device=dev), torch.as_tensor(f_s, device=dev),
                     torch.as_tensor(m_s, device=dev), None, npix, npix, 0.45 / 3.0e5,
                     0.45 / 3.0e5, 1e-7, True)
    chans = np.arange(224, 256)
    obs = simulation.device_observation(400, 32, 50e6, 350e6, config="LOW", device=dev,
                                        nchan_total=256, channels=chans)
    nvis = obs["nrow"] * 32
    assert nvis == 1_674_444_800
    cell = 0.25 / obs["umax"]
    d, info = kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], npix, npix, cell,
                               cell, 1e-7, True, flip_uw=True)
    assert info["ngrid_x"] == 2 * npix and info["nplanes"] > 40
    # exact sums at 12 pixels (host copies of the shard: 13.4 GB of c64)
    rng = np.random.default_rng(41)
    px = np.concatenate([[npix // 2, npix // 2 + 3], rng.integers(npix // 8, 7 * npix // 8, 10)])
    py = np.concatenate([[npix // 2, npix // 2 - 5], rng.integers(npix // 8, 7 * npix // 8, 10)])
    uvw_h = obs["uvw"].cpu().numpy() * FLIP_UW
    freq_h = obs["freq"].cpu().numpy()
    ex = wgrid_cpu.exact_pixels(uvw_h, freq_h, obs["vis"].cpu().numpy(), None, npix, npix, cell,
                                cell, True, px, py, nthreads=_threads())
    e_px = rel_rms(d.cpu().numpy()[px, py], ex)
    # adjointness with a random sparse image
    y = torch.zeros((npix, npix), dtype=torch.float64, device=dev)
    iy = rng.integers(npix // 4, 3 * npix // 4, (2, 4096))
    y[iy[0], iy[1]] = torch.as_tensor(rng.normal(size=4096), device=dev)
    v, _ = kernels.dirty2ms(obs["uvw"], obs["freq"], y, obs["wgt"], cell, cell, 1e-7, True,
                            flip_uw=True)
    lhs = float(torch.sum(d * y))
    rhs = 0.0
    for a in range(0, obs["nrow"], 4_000_000):
        vv = v[a:a + 4_000_000].to(torch.complex128)
        xx = obs["vis"][a:a + 4_000_000].to(torch.complex128)
        rhs += float(torch.sum((vv.conj() * xx).real))
    e_adj = abs(lhs - rhs) / abs(lhs)
    del v
    # unit point source off the phase centre
    x0, y0 = npix // 2 + 1200, npix // 2 - 700
    pt = torch.zeros_like(y)
    pt[x0, y0] = 1.0
    l0, m0 = (x0 - npix // 2) * cell, (y0 - npix // 2) * cell
    n0 = math.sqrt(1.0 - l0 * l0 - m0 * m0)
    vp, _ = kernels.dirty2ms(obs["uvw"], obs["freq"], pt, None, cell, cell, 1e-7, True,
                             flip_uw=True)
    e_amp = 0.0
    for a in range(0, obs["nrow"], 4_000_000):
        e_amp = max(e_amp, float(torch.max(torch.abs(torch.abs(vp[a:a + 4_000_000]) * n0 - 1.0))))
    dp, _ = kernels.ms2dirty(obs["uvw"], obs["freq"], vp, None, npix, npix, cell, cell, 1e-7,
                             True, flip_uw=True)
    k = int(torch.argmax(dp))
    peak = float(dp.view(-1)[k]) * n0 * n0 / nvis
    del vp, dp
    # the benchmarked streamed form: 3 channel batches through one set of
    # resident planes (the merged bounds give the single call's layout)
    blocks = [(0, 11), (11, 22), (22, 32)]
    b = kernels.merge_bounds(*[kernels.uvw_bounds(obs["uvw"], obs["freq"][a:e]) for a, e in blocks])
    db = None
    for i, (a, e) in enumerate(blocks):
        db, binfo = kernels.ms2dirty_batch(obs["uvw"], obs["freq"][a:e],
                                           obs["vis"][:, a:e].contiguous(),
                                           obs["wgt"][:, a:e].contiguous(), npix, npix, cell, cell,
                                           b, first=i == 0, last=i == len(blocks) - 1,
                                           epsilon=1e-7, flip_uw=True)
        assert binfo["nplanes"] == info["nplanes"] and binfo["w0"] == info["w0"]
    e_batch = float(torch.sqrt(torch.mean((db - d) ** 2) / torch.mean(d ** 2)))
    e_bpx = rel_rms(db.cpu().numpy()[px, py], ex)
    # the cached workspace leaves the caller room: 16 GiB from torch
    big = torch.empty(16 << 30, dtype=torch.uint8, device=dev)
    del big
    print(f"\nC4 shard (1.67 Gvis, {info['nplanes']} planes, 16384^2 grid): exact pixels rel-RMS "
          f"{e_px:.2e}; adjointness {e_adj:.2e}; point source max||V| n - 1| {e_amp:.2e}, "
          f"peak at {(k // npix, k % npix)} value n^2/sum(w) x {peak:.8f}; 3 batches vs single "
          f"call {e_batch:.2e}, vs exact pixels {e_bpx:.2e}")
    # (fp32 sums in another order: each side is ~1.3e-6 from the exact sums)
    assert e_batch < 5e-6 and e_bpx < TOL
    assert (k // npix, k % npix) == (x0, y0)
    assert abs(peak - 1.0) < 1e-5
    assert e_amp < 1e-5
    assert e_adj < 5e-6
    assert e_px < TOL


def _c4_band(dev):
    """C4's rows (SKA-LOW 512 stations x 400 times, uvw resident), the band's
    256 frequencies and the cell -- bench.py run_c4's setup."""
    from ska_sdp_func_python_amd import simulation
    obs = simulation.device_observation(400, 1, 50e6, 350e6, config="LOW", device=dev,
                                        nchan_total=256, channels=[0])
    del obs["vis"], obs["wgt"]
    return obs["uvw"], obs["nrow"], np.linspace(50e6, 350e6, 256), 0.25 / obs["umax"]


def _point_vis(uvw, freq, l0, m0, rows=2_000_000):
    """Visibilities of a unit point source at (l0, m0) in the ducc0 frame of
    an invert with flip_uw (u, w negated): dirty[x0, y0] = sum(w) / n0."""
    n0 = math.sqrt(1.0 - l0 * l0 - m0 * m0)
    out = torch.empty((uvw.shape[0], freq.shape[0]), dtype=torch.complex64, device=uvw.device)
    s = freq.to(torch.float64)[None, :] / 299792458.0
    for a in range(0, uvw.shape[0], rows):
        u = uvw[a:a + rows]
        d = (-u[:, 0:1] * l0 + u[:, 1:2] * m0 + u[:, 2:3] * (n0 - 1.0)) * s
        d = d - torch.round(d)
        out[a:a + rows] = torch.polar(torch.ones_like(d), -2.0 * math.pi * d).to(torch.complex64)
    return out


def _c4_streamed_checks(tag, uvw, freqs, batches, vis_of, npix, cell, npx=32, ncpu=4, seed=90,
                        px_tol=2e-6, adj_tol=5e-6, peak_tol=1e-5):
    """The streamed (sdp_hip_ms2dirty_batch) invert of `batches` against
    exact direct sums at `npx` sampled pixels, adjointness <A x, y> = Re <x,
    A^H y> over every visibility, and a unit point source (peak pixel and
    value sum(w)/n0).  The exact sums: the fp64 torch restatement on the
    device (gpu_helpers.exact_pixels_dev) at all pixels, pinned to the C
    oracle (oracle/wgrid_cpu.c, accumulated per batch on the host) at the
    first `ncpu` of them (agreement 1e-10)."""
    import wgrid_cpu
    from gpu_helpers import exact_pixels_dev
    from ska_sdp_func_python_amd import kernels, parallel
    dev = uvw.device
    f_all = torch.as_tensor(freqs, device=dev)
    nvis = uvw.shape[0] * sum(e - a for a, e in batches)
    d = parallel.invert_batched_shard(uvw, f_all, vis_of, batches, npix, cell, 1e-7, True,
                                      flip_uw=True)  # RASCIL [y, x]
    print(f"\n{tag}: streamed invert of {nvis / 1e9:.2f} Gvis in {len(batches)} batches done",
          flush=True)
    rng = np.random.default_rng(seed)
    px = np.concatenate([[npix // 2], rng.integers(npix // 8, 7 * npix // 8, npx - 1)])
    py = np.concatenate([[npix // 2 - 3], rng.integers(npix // 8, 7 * npix // 8, npx - 1)])
    uvw_h = uvw.cpu().numpy() * FLIP_UW
    flip = torch.as_tensor(FLIP_UW, device=dev)
    ex = np.zeros(npx)
    ex_cpu = np.zeros(ncpu)
    for i, (a, e) in enumerate(batches):
        vis_d = vis_of(a, e)
        ex += exact_pixels_dev(uvw * flip, freqs[a:e], vis_d, npix, cell, px, py)
        vis_h = vis_d.cpu().numpy()
        del vis_d
        ex_cpu += wgrid_cpu.exact_pixels(uvw_h, freqs[a:e], vis_h, None, npix, npix, cell, cell,
                                         True, px[:ncpu], py[:ncpu], nthreads=_threads())
        del vis_h
        print(f"{tag}: exact pixels, batch {i + 1}/{len(batches)}", flush=True)
    e_pin = rel_rms(ex[:ncpu], ex_cpu)
    e_px = rel_rms(d.cpu().numpy()[py, px], ex)
    # adjointness: a random sparse model (ducc0 [x, y]) degridded batch by batch
    y = torch.zeros((npix, npix), dtype=torch.float64, device=dev)
    iy = rng.integers(npix // 4, 3 * npix // 4, (2, 4096))
    y[iy[0], iy[1]] = torch.as_tensor(rng.normal(size=4096), device=dev)
    lhs = float(torch.sum(d.T * y))
    rhs = 0.0
    for a, e in batches:
        v, _ = kernels.dirty2ms(uvw, f_all[a:e], y, None, cell, cell, 1e-7, True, flip_uw=True)
        x = vis_of(a, e)
        for r in range(0, uvw.shape[0], 4_000_000):
            rhs += float(torch.sum((v[r:r + 4_000_000].to(torch.complex128).conj()
                                    * x[r:r + 4_000_000].to(torch.complex128)).real))
        del v, x
    e_adj = abs(lhs - rhs) / abs(lhs)
    # the predicts' outputs sit in torch's cache and their bucketing in the
    # library's workspace: give the next streamed invert's 71 planes the room
    torch.cuda.empty_cache()
    kernels.release_workspace()
    # unit point source off the phase centre
    x0, y0 = npix // 2 + 1200, npix // 2 - 700
    l0, m0 = (x0 - npix // 2) * cell, (y0 - npix // 2) * cell
    n0 = math.sqrt(1.0 - l0 * l0 - m0 * m0)
    dp = parallel.invert_batched_shard(uvw, f_all,
                                       lambda a, e: _point_vis(uvw, f_all[a:e], l0, m0), batches,
                                       npix, cell, 1e-7, True, flip_uw=True)
    k = int(torch.argmax(dp))
    peak = float(dp.view(-1)[k]) * n0 / nvis
    print(f"{tag}: {npx} exact pixels rel-RMS {e_px:.2e} (device sums vs the C oracle at {ncpu}: "
          f"{e_pin:.1e}); adjointness {e_adj:.2e}; point source peak at (y, x) "
          f"{(k // npix, k % npix)} value n0/sum(w) x {peak:.8f}", flush=True)
    assert e_pin < 1e-10
    assert e_px < px_tol
    assert e_adj < adj_tol
    assert (k // npix, k % npix) == (y0, x0)
    assert abs(peak - 1.0) < peak_tol


@pytest.mark.timeout(1800)
def test_c4_full_band_streamed_as_benchmarked():
    """The c4_n1 object's exact form: all 256 channels of the SKA-LOW band
    (13.4 Gvis) streamed through sdp_hip_ms2dirty_batch in bench.py's 8
    channel batches (generated on device per batch, run_c4's seeds) into the
    band's 71 resident 16384^2 planes, against exact sums, adjointness and a
    point source -- the reference's per-channel loop (ng.py:259-289) gridded
    as one streamed invert."""
    dev = torch.device("cuda:0")
    uvw, nrow, freqs, cell = _c4_band(dev)
    nb = max(-(-256 // 40), math.ceil(nrow * 256 / 1.8e9))
    assert nb == 8
    cuts = [256 * i // nb for i in range(nb + 1)]
    batches = list(zip(cuts[:-1], cuts[1:]))
    gen = torch.Generator(device=dev)

    def vis_of(a, e):
        gen.manual_seed(a)
        return torch.randn((nrow, e - a), generator=gen, device=dev, dtype=torch.complex64)

    # the dense uv core's cells take ~10^6-10^7 flushed additions over the
    # whole band: they accumulate in the fp64 companion planes (CoreAcc,
    # csrc/wstack.hip), so the band holds the same bounds as one shard
    # (round 4, all-fp32 planes: exact pixels 2.5e-6 / 5.6e-6, adjointness
    # 5.3e-5 / 6.1e-5, run to run with the atomics' order)
    _c4_streamed_checks("C4 full band", uvw, freqs, batches, vis_of, 8192, cell,
                        adj_tol=1e-5)


@pytest.mark.timeout(1500)
def test_c4_largest_w_rank_of_the_8way_row_partition():
    """Rank 7 of bench.py's default 8-GPU C4 partition (rows by w,
    parallel.wrow_partition: the interval of the largest |w|, all 256
    channels, its own plane layout) at full size, as run_c4 streams it."""
    from ska_sdp_func_python_amd import kernels, parallel
    dev = torch.device("cuda:0")
    uvw, nrow, freqs, cell = _c4_band(dev)
    f_all = torch.as_tensor(freqs, device=dev)
    lay = kernels.wstack_layout(kernels.uvw_bounds(uvw, f_all), 8192, 8192, cell, cell, 1e-7, True,
                                flip_uw=True)
    order, cuts, _ = parallel.wrow_partition((-uvw[:, 2]).cpu().numpy(), freqs, 8, lay["dw"],
                                             lay["support"])
    rows = torch.as_tensor(order[cuts[7]:cuts[8]], device=dev)
    u7 = uvw[rows].contiguous()
    del uvw, rows
    n7 = u7.shape[0]
    nb = max(1, math.ceil(n7 * 256 / 1.8e9))
    cb = [256 * i // nb for i in range(nb + 1)]
    batches = list(zip(cb[:-1], cb[1:]))
    gen = torch.Generator(device=dev)

    def vis_of(a, e):
        gen.manual_seed(7919 * 7 + a)
        return torch.randn((n7, e - a), generator=gen, device=dev, dtype=torch.complex64)

    _c4_streamed_checks(f"C4 wrow rank 7/8 ({n7} rows)", u7, freqs, batches, vis_of, 8192, cell,
                        adj_tol=5e-6)


# ---------------------------------------------------------------------------
# C5: StefCal 512 stations x 256 channels x 1000 times
# ---------------------------------------------------------------------------
@pytest.mark.timeout(900)
def test_c5_full_batch_and_sampled_rows():
    """All 256,000 (time, channel) solves of C5 (B jones: per-channel gains,
    one convergence test per time row over its 256 channels, as in the
    reference's solvers.py:268) in batches of 16 time rows, against the true
    gains (x_b = g_a1 conj(g_a2), unit weights); then 8 rows drawn from the
    same distribution (512 stations x 32 channels, noise 1e-3, random
    weights) against the restated reference solver
    (oracle/ref_oracle.stefcal_row): the same iteration count and gains
    within 1e-7."""
    import ref_oracle as ro
    from ska_sdp_func_python_amd import kernels
    nants, nchan, ntime, batch = 512, 256, 1000, 16
    dev = torch.device("cuda:0")
    a1, a2 = np.triu_indices(nants, 1)
    perm, conj, rs, ant2 = kernels.canonical_baselines(a1, a2, nants)
    a1t, a2t = torch.as_tensor(a1[perm], device=dev), torch.as_tensor(a2[perm], device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1805550721)
    worst, worst_res, iters = 0.0, 0.0, []
    for t0 in range(0, ntime, batch):
        nt = min(batch, ntime - t0)
        amp = torch.exp(0.1 * torch.randn((nt, nants, nchan), generator=gen, device=dev,
                                          dtype=torch.float64))
        g = torch.polar(amp, 0.1 * torch.randn((nt, nants, nchan), generator=gen, device=dev,
                                               dtype=torch.float64))
        xb = (g[:, a1t, :] * torch.conj(g[:, a2t, :]))[..., None].contiguous()
        wb = torch.ones(xb.shape, dtype=torch.float64, device=dev)
        gain = torch.ones((nt, nants, nchan, 1, 1), dtype=torch.complex128, device=dev)
        gwt = torch.zeros((nt, nants, nchan, 1, 1), dtype=torch.float64, device=dev)
        res, used = kernels.solve_gains(xb, wb, gain, gwt, rs, ant2, mode=0, niter=200, tol=1e-6,
                                        phase_only=False)
        est = gain[..., 0, 0]
        est = est * torch.conj(est[:, :1]) / torch.abs(est[:, :1])
        tru = g * torch.conj(g[:, :1]) / torch.abs(g[:, :1])
        worst = max(worst, float(torch.max(torch.abs(est - tru))))
        worst_res = max(worst_res, float(res.max()))
        iters.append(int(used.max()))
        del xb, wb, g, gain, gwt
    rng = np.random.default_rng(1805550721)
    nch = 32
    dg_max, it_pairs = 0.0, []
    for row in range(8):
        g = rng.lognormal(0, 0.1, (nants, nch)) * np.exp(1j * rng.normal(0, 0.1, (nants, nch)))
        xb = (g[a1] * np.conj(g[a2]))[..., None]
        xb = xb + 1e-3 * (rng.normal(size=xb.shape) + 1j * rng.normal(size=xb.shape))
        wb = rng.uniform(0.5, 1.5, xb.shape)
        gain = torch.ones((1, nants, nch, 1, 1), dtype=torch.complex128, device=dev)
        gwt = torch.zeros((1, nants, nch, 1, 1), dtype=torch.float64, device=dev)
        res, used = kernels.solve_gains(torch.as_tensor(xb[None, perm], device=dev),
                                        torch.as_tensor(wb[None, perm], device=dev), gain, gwt,
                                        rs, ant2, mode=0, niter=200, tol=1e-6, phase_only=False)
        eg, ew, er, eu = ro.stefcal_row(xb, wb, list(zip(a1, a2)), nants,
                                        np.ones((nants, nch, 1, 1), complex),
                                        np.zeros((nants, nch, 1, 1)), niter=200, tol=1e-6,
                                        phase_only=False)
        it_pairs.append((int(used[0]), eu))
        dg_max = max(dg_max, float(np.max(np.abs(gain[0].cpu().numpy() - eg))))
        np.testing.assert_allclose(gwt[0].cpu().numpy(), ew, rtol=1e-6)
        np.testing.assert_allclose(res[0].cpu().numpy(), er, rtol=1e-5)
    print(f"\nC5 256,000 solves: max gain error vs truth {worst:.2e}, max residual "
          f"{worst_res:.2e}, iterations max {max(iters)}; 8 sampled rows vs oracle: iterations "
          f"{it_pairs}, max|dgain| {dg_max:.2e}")
    assert worst < 1e-5 and worst_res < 1e-6 and max(iters) < 200
    assert all(a == b for a, b in it_pairs)
    assert dg_max < 1e-7
