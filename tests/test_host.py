"""CPU: host-side logic of the product package (no GPU compute)."""

import math
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def test_library_exports_every_header_symbol():
    from ska_sdp_func_python_amd import _lib
    with open(os.path.join(ROOT, "include", "ska_sdp_hip.h")) as f:
        declared = set(re.findall(r"^\s*int\s+(sdp_hip_\w+)\s*\(", f.read(), re.M))
    assert declared, "no declarations parsed"
    lib = _lib.load()
    missing = [s for s in sorted(declared) if not hasattr(lib, s)]
    assert not missing, missing
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    assert lib.sdp_hip_version() >= 1


def test_library_reports_errors_without_device():
    from ska_sdp_func_python_amd import _lib
    import ctypes
    n = ctypes.c_int(-1)
    _lib.call("sdp_hip_device_count", ctypes.byref(n))
    assert n.value >= 0


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ska_sdp_func_python_amd import _device, _lib
    with pytest.raises(_lib.HipLibraryError):
        _device.device()


def test_skycoord_to_lmn_known_answer():
    """reference tests/imaging/test_dft_skycomponent_visibility.py:165-167."""
    from ska_sdp_func_python_amd.datamodels import SkyCoord
    from ska_sdp_func_python_amd.util.coordinate_support import skycoord_to_lmn
    l, m, n = skycoord_to_lmn(SkyCoord(181.0, -35.0, unit="deg"), SkyCoord(180.0, -35.0, unit="deg"))
    np.testing.assert_allclose([l, m, n], [1.42961744e-02, -7.15598688e-05, -1.02198084e-04],
                               rtol=1e-7)


def test_pol_conversion_round_trip_and_known_values():
    from ska_sdp_func_python_amd.datamodels import PolarisationFrame as PF, convert_pol_frame
    iquv = np.array([[100.0, 20.0, -10.0, 1.0]])
    lin = convert_pol_frame(iquv, PF("stokesIQUV"), PF("linear"))
    np.testing.assert_allclose(lin, [[120, -10 + 1j, -10 - 1j, 80]])
    back = convert_pol_frame(lin, PF("linear"), PF("stokesIQUV"))
    np.testing.assert_allclose(back, iquv, atol=1e-12)
    circ = convert_pol_frame(iquv, PF("stokesIQUV"), PF("circular"))
    np.testing.assert_allclose(convert_pol_frame(circ, PF("circular"), PF("stokesIQUV")), iquv,
                               atol=1e-12)
    with pytest.raises(ValueError):
        convert_pol_frame(iquv, PF("stokesIQUV"), PF("linearnp"))


def test_canonical_baselines():
    from ska_sdp_func_python_amd.kernels import canonical_baselines
    a1 = np.array([0, 2, 1, 3, 1, 2])
    a2 = np.array([1, 0, 1, 1, 2, 3])
    perm, conj, rs, ant2 = canonical_baselines(a1, a2, 4)
    pairs = [(min(a1[p], a2[p]), max(a1[p], a2[p])) for p in perm]
    assert pairs == [(0, 1), (0, 2), (1, 2), (1, 3), (2, 3)]
    assert list(conj) == [False, True, False, True, False]
    assert list(rs) == [0, 2, 4, 5, 5] and list(ant2) == [1, 2, 2, 3, 3]


def test_shard_ranges_cover():
    from ska_sdp_func_python_amd.parallel import shard_range
    for n in (1, 7, 64, 100):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                lo, hi = shard_range(n, r, world)
                got.extend(range(lo, hi))
            assert got == list(range(n))


def test_synthetic_layouts():
    from ska_sdp_func_python_amd import simulation as s
    mid = s.ska_mid_layout()
    low = s.ska_low_layout()
    assert mid.shape == (197, 2) and low.shape == (512, 2)
    assert 60e3 < np.hypot(*mid.T).max() < 80e3
    assert 30e3 < np.hypot(*low.T).max() < 40e3
    vis = s.make_visibility("MID", nants=7, ntimes=10)
    assert vis.vis.shape == (10, 21, 1, 1)


def test_wcs_and_image_centre():
    from ska_sdp_func_python_amd.datamodels import SkyCoord, create_image, pixel_to_skycoord
    pc = SkyCoord(180.0, -45.0, unit="deg")
    im = create_image(256, 1e-4, pc)
    c = pixel_to_skycoord(129, 129, im.image_acc.wcs, origin=1)
    assert pc.separation(c).rad < 1e-15
    east = pixel_to_skycoord(128, 129, im.image_acc.wcs, origin=1)  # one pixel left = east
    assert east.ra.rad > pc.ra.rad
    assert abs(im.image_acc.wcs.sub([4]).wcs_world2pix(np.array([1e8]), 0)[0][0]) < 1e-12


def test_skycoord_pixel_round_trip_and_apply_beam():
    """skycoord_to_pixel inverts pixel_to_skycoord (SIN, origin 1); the
    reference's apply_beam_to_skycomponent rules (sky_component/operations.py:
    411-425): flux x beam at the rounded pixel, / beam for inverse, zero off
    the image."""
    import math
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.sky_component import apply_beam_to_skycomponent
    pc = dm.SkyCoord(math.radians(30.0), math.radians(-40.0))
    im = dm.create_image(64, 0.002, pc)
    for x, y in ((33.0, 33.0), (10.25, 50.5), (60.0, 3.0)):
        c = dm.pixel_to_skycoord(x, y, im.image_acc.wcs, origin=1)
        px, py = dm.skycoord_to_pixel(c, im.image_acc.wcs, origin=1)
        assert abs(px[0] - x) < 1e-9 and abs(py[0] - y) < 1e-9
    im["pixels"].data[0, 0] = np.arange(64 * 64, dtype=float).reshape(64, 64) + 1.0
    comps = [dm.SkyComponent(dm.pixel_to_skycoord(20.0, 30.0, im.image_acc.wcs), [1e8], flux=[[2.0]]),
             dm.SkyComponent(dm.pixel_to_skycoord(200.0, 30.0, im.image_acc.wcs), [1e8], flux=[[2.0]])]
    out = apply_beam_to_skycomponent(comps, im)
    # the reference indexes the beam with the 1-relative pixel coordinates
    # (origin=1) as they are: pixel (20, 30) reads data[..., 30, 20]
    assert out[0].flux[0, 0] == 2.0 * im["pixels"].data[0, 0, 30, 20]
    assert out[1].flux[0, 0] == 0.0
    inv = apply_beam_to_skycomponent(comps[0], im, inverse=True)
    assert inv.flux[0, 0] == 2.0 / im["pixels"].data[0, 0, 30, 20]


def test_unknown_imaging_context_raises():
    """reference imaging/imaging.py:55, :105: an unknown context is a ValueError
    (raised before any device work)."""
    from ska_sdp_func_python_amd.imaging import invert_visibility, predict_visibility
    with pytest.raises(ValueError, match="Unknown imaging context"):
        invert_visibility(None, None, context="wstack-nope")
    with pytest.raises(ValueError, match="Unknown imaging context"):
        predict_visibility(None, None, context="")


def test_cf_channel_map_checked_like_numpy_indexing():
    """vis -> image channels past the GridData's / CF's channel axis raise
    IndexError (the reference's gd[imchan], grid_data/gridding.py:226-245);
    the check runs on the host before any launch."""
    import torch
    from ska_sdp_func_python_amd import kernels
    nrow, nchan, npol = 5, 3, 1
    maps = {k: torch.zeros((nchan, nrow), dtype=torch.int32) for k in ("pu", "pv", "pwc", "pdu", "pdv")}
    vis = torch.zeros((nrow, nchan, npol), dtype=torch.complex128)
    wt = torch.ones((nrow, nchan, npol), dtype=torch.float64)
    cf = torch.zeros((2, npol, 1, 1, 1, 4, 4), dtype=torch.complex128)
    grid = torch.zeros((2, npol, 16, 16), dtype=torch.complex128)
    sumwt = torch.zeros((2, npol), dtype=torch.float64)
    for bad in ([0, 1, 2], [0, -3, 1]):
        with pytest.raises(IndexError):
            kernels.grid_cf(maps, torch.tensor(bad, dtype=torch.int32), vis, wt, cf, grid, sumwt)
        with pytest.raises(IndexError):
            kernels.degrid_cf(maps, torch.tensor(bad, dtype=torch.int32), grid, cf, nrow, nchan,
                              torch.zeros((nrow, nchan, npol), dtype=torch.complex128))
    with pytest.raises(ValueError, match="pol axes"):
        kernels.degrid_cf(maps, torch.zeros(nchan, dtype=torch.int32),
                          torch.zeros((2, 2, 16, 16), dtype=torch.complex128), cf, nrow, nchan,
                          torch.zeros((nrow, nchan, npol), dtype=torch.complex128))
    with pytest.raises(ValueError, match="out must be"):
        kernels.degrid_cf(maps, torch.zeros(nchan, dtype=torch.int32), grid, cf, nrow, nchan,
                          torch.zeros((nrow, nchan, npol), dtype=torch.complex64))


def test_epsilon_below_fp32_floor_is_reported_once(caplog):
    """epsilon < 1e-7 selects the fp64 NUFFT (no flag bits, no note);
    precision="fp32" serves it at the fp32 floor (SDP_HIP_FP32) and says so
    once per process; an unknown precision is refused."""
    import logging
    import torch
    from ska_sdp_func_python_amd import _lib, kernels
    kernels._eps_warned = False
    assert kernels._prec_bits(1e-12) == 0 and kernels._prec_bits(1e-6, "fp32") == 0
    with caplog.at_level(logging.WARNING, logger="func-python-logger"):
        for _ in range(2):
            assert kernels._prec_bits(1e-12, "fp32") == _lib.SDP_HIP_FP32
    msgs = [r.getMessage() for r in caplog.records if "floor epsilon" in r.getMessage()]
    assert len(msgs) == 1 and "1.0e-12" in msgs[0]
    with pytest.raises(ValueError):
        kernels._prec_bits(1e-12, "fp16")
    uvw = torch.zeros((4, 3), dtype=torch.float64)
    with pytest.raises(ValueError):  # host tensors are rejected
        kernels.ms2dirty(uvw, torch.ones(1), None, None, 8, 8, 1e-3, 1e-3, 1e-12,
                         precision="fp32")


def test_balanced_channel_blocks_cover_and_balance():
    """The C4 strong-scaling partition: contiguous, covering, and within 3 % of
    the mean modelled cost at 2/4/8 ranks (parallel.balanced_channel_blocks)."""
    from ska_sdp_func_python_amd import parallel
    f = np.linspace(50e6, 350e6, 256)
    for world in (1, 2, 3, 4, 8):
        b = parallel.balanced_channel_blocks(f, world)
        assert len(b) == world and b[0][0] == 0 and b[-1][1] == 256
        assert all(b[i][1] == b[i + 1][0] and b[i][0] < b[i][1] for i in range(world - 1))
        c = [parallel.c4_block_cost(f[a:e]) for a, e in b]
        assert max(c) <= 1.03 * (sum(c) / world)


def test_wslab_partition_covers_the_planes_and_balances():
    """parallel.wslab_partition: contiguous first-plane slabs covering the
    layout, none empty while there are planes enough, the modelled costs
    balanced within one plane's worth of work; more ranks than planes leave
    the extra ranks empty.  first_plane_histogram matches the bucketing's
    first-plane formula on CPU tensors."""
    import numpy as np
    import torch
    from ska_sdp_func_python_amd import parallel
    rng = np.random.default_rng(7)
    hist = rng.gamma(0.6, 1e7, 71)
    hist[:10] *= 8.0  # the dense low-|w| planes
    for world in (1, 2, 4, 8):
        slabs = parallel.wslab_partition(hist, world, 8)
        assert len(slabs) == world and slabs[0][0] == 0 and slabs[-1][1] == 71
        assert all(s[1] == t[0] and s[0] < s[1] for s, t in zip(slabs, slabs[1:]))
        costs = [parallel.wslab_cost(hist, a, e, 8, hist.sum()) for a, e in slabs]
        best_single = max(parallel.wslab_cost(hist, p, p + 1, 8, hist.sum()) for p in range(71))
        assert max(costs) <= max(best_single, sum(costs) / world + 3 * parallel.WSLAB_PLANE_MS
                                 + parallel.WSLAB_VIS_MS_PER_G * hist.max() / 1e9)
    few = parallel.wslab_partition(np.ones(3), 5, 8)
    assert few[:3] == [(0, 1), (1, 2), (2, 3)] and few[3:] == [(3, 3), (3, 3)]
    uvw = torch.as_tensor(rng.normal(size=(500, 3)) * 300.0)
    freqs = np.array([1.0e8, 1.5e8, 2.0e8])
    lay = {"nps": 40, "support": 8, "w0": -80.0, "dw": 4.0}
    h = parallel.first_plane_histogram(uvw, freqs, lay, flip_uw=True)
    w = -uvw[:, 2].numpy()
    ref = np.zeros(40)
    for f in freqs:
        p0 = np.floor(np.clip((w * f / 299792458.0 + 80.0) / 4.0 - 4.0, -2, 2e9)).astype(int) + 1
        np.add.at(ref, np.clip(p0, 0, 39), 1)
    assert np.array_equal(h, ref)


def test_wrow_partition_covers_the_rows_and_balances():
    """parallel.wrow_partition: rank r owns rows order[cuts[r]:cuts[r+1]], a
    contiguous interval of w; the intervals cover all rows, the modelled
    costs are balanced, and the small-|w| ranks hold fewer planes."""
    import numpy as np
    from ska_sdp_func_python_amd import parallel
    rng = np.random.default_rng(3)
    w = np.concatenate([rng.normal(0, 30.0, 200000), rng.normal(0, 800.0, 40000)])
    f = np.linspace(50e6, 350e6, 256)
    for world in (1, 2, 4, 8):
        # (vis costs scaled x1000: the 240k rows stand for a C4-sized band)
        order, cuts, costs = parallel.wrow_partition(w, f, world, 1734.0, 8, vis_ms_per_g=65.1e3,
                                                     vis_w_ms_per_g=53.7e3)
        assert len(cuts) == world + 1 and cuts[0] == 0 and cuts[-1] == w.size
        assert all(a <= b for a, b in zip(cuts, cuts[1:]))
        ws = w[order]
        assert np.all(np.diff(ws) >= 0)
        if world > 1:
            assert max(costs) < 1.1 * min(costs) + 2 * parallel.WROW_PLANE_MS
            pl = [parallel.wrow_planes(ws[a], ws[e - 1], f.min(), f.max(), 1734.0, 8)
                  for a, e in zip(cuts[:-1], cuts[1:])]
            mid = world // 2
            assert pl[mid] <= max(pl[0], pl[-1])


def test_groupby_time_groups_distinct_sorted_times():
    """Visibility.groupby("time") follows xarray: one group per distinct time
    value, in increasing order, holding every row with that time (repeated
    and unsorted time stamps included)."""
    import numpy as np
    from ska_sdp_func_python_amd import datamodels as dm
    times = np.array([3.0, 1.0, 3.0, 2.0, 2.0])
    nt, nb = len(times), 3
    vis = dm.Visibility.constructor(
        frequency=np.array([1e9]), channel_bandwidth=np.array([1e6]),
        phasecentre=dm.SkyCoord(0.0, -0.5), uvw=np.arange(nt * nb * 3, dtype=float).reshape(nt, nb, 3),
        time=times, vis=np.arange(nt * nb, dtype=complex).reshape(nt, nb, 1, 1),
        baselines=np.stack(np.triu_indices(3, 1), 1))
    groups = vis.groupby("time", squeeze=False)
    assert [t for t, _ in groups] == [1.0, 2.0, 3.0]
    rows = {1.0: [1], 2.0: [3, 4], 3.0: [0, 2]}
    for t, g in groups:
        np.testing.assert_array_equal(np.asarray(g.time.data), [t] * len(rows[t]))
        np.testing.assert_array_equal(np.asarray(g.vis.data)[:, :, 0, 0],
                                      np.arange(nt * nb).reshape(nt, nb)[rows[t]])


def test_groupby_time_skips_non_finite_times():
    """A row with a NaN (or infinite) time belongs to no group, as xarray's
    groupby drops NaN labels; the finite times still group as usual."""
    import numpy as np
    from ska_sdp_func_python_amd import datamodels as dm
    times = np.array([3.0, np.nan, 1.0, 3.0, np.inf, 2.0])
    nt, nb = len(times), 3
    vis = dm.Visibility.constructor(
        frequency=np.array([1e9]), channel_bandwidth=np.array([1e6]),
        phasecentre=dm.SkyCoord(0.0, -0.5), uvw=np.zeros((nt, nb, 3)),
        time=times, vis=np.arange(nt * nb, dtype=complex).reshape(nt, nb, 1, 1),
        baselines=np.stack(np.triu_indices(3, 1), 1))
    groups = vis.groupby("time", squeeze=False)
    assert [t for t, _ in groups] == [1.0, 2.0, 3.0]
    rows = {1.0: [2], 2.0: [5], 3.0: [0, 3]}
    for t, g in groups:
        np.testing.assert_array_equal(np.asarray(g.vis.data)[:, :, 0, 0],
                                      np.arange(nt * nb).reshape(nt, nb)[rows[t]])
