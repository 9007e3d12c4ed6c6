"""GPU parity of the calibration neighbours of StefCal
through the C ABI: apply_gaintable against the reference-generated fixtures
(tests/golden/applygt_*.npz, rtol 1e-12: fp64 with numpy's complex division;
LAPACK's 2x2 inverse and BLAS products differ only in rounding), and
divide_visibility / the solver's point-source sums against
oracle/calops_oracle.py."""

import numpy as np
import pytest
import torch

import calops_oracle as co
from conftest import golden
from gpu_helpers import vis_from_arrays

pytestmark = pytest.mark.gpu
TAGS = ["p1", "p1_g1chan", "p2", "p4", "p4_circ_g1chan"]


def _objects(g, device):
    from ska_sdp_func_python_amd import datamodels as dm
    pf = str(g["pol_frame"])
    nt = len(g["time"])
    vis = vis_from_arrays(np.zeros((nt, len(g["baselines"]), 3)), np.linspace(1e8, 1.1e8, g["vis"].shape[2]),
                          g["vis"].copy(), weight=g["weight"].copy(), flags=g["flags"].copy(),
                          baselines=g["baselines"], pf=pf, times=g["time"])
    if device:
        for name in ("vis", "weight", "flags"):
            vis[name] = torch.as_tensor(np.asarray(vis[name].data), device="cuda")
    nrec = g["gain"].shape[-1]
    gt = dm.GainTable.constructor(g["gain"].copy(), g["gt_time"], g["gt_interval"],
                                  np.ones(g["gain"].shape), np.zeros(g["gain"].shape[:1] + g["gain"].shape[2:]),
                                  np.linspace(1e8, 1.1e8, g["gain"].shape[2]),
                                  dm.PolarisationFrame("stokesI" if nrec == 1 else pf))
    return vis, gt


@pytest.mark.parametrize("device", [False, True])
@pytest.mark.parametrize("tag", TAGS)
def test_apply_gaintable_matches_reference(tag, device):
    from ska_sdp_func_python_amd.calibration import apply_gaintable
    g = golden(f"applygt_{tag}.npz")
    for inverse in (False, True):
        for use_flags in (False, True):
            vis, gt = _objects(g, device)
            out = apply_gaintable(vis, gt, inverse=inverse, use_flags=use_flags)
            assert out is vis
            k = f"i{int(inverse)}_f{int(use_flags)}"
            v, w = out["vis"].data, out["weight"].data
            if device:
                v, w = v.cpu().numpy(), w.cpu().numpy()
            np.testing.assert_allclose(v, g[f"vis_{k}"], rtol=1e-12, atol=1e-14, err_msg=k)
            np.testing.assert_array_equal(w, g[f"wt_{k}"], err_msg=k)


def test_apply_gaintable_overlapping_windows_sequential():
    """A vis time inside two gain rows' windows gets both, one after the other
    (the reference's row loop, operations.py:55-61)."""
    from ska_sdp_func_python_amd.calibration import apply_gaintable
    g = golden("applygt_p4.npz")
    vis, gt = _objects(g, False)
    gt["interval"].data[...] = 3.0 * gt["interval"].data
    expect_v, expect_w = co.apply_gaintable(g["vis"], g["weight"], g["flags"], g["time"], g["baselines"],
                                            g["gain"], g["gt_time"], gt["interval"].data, False, False)
    out = apply_gaintable(vis, gt)
    np.testing.assert_allclose(out["vis"].data, expect_v, rtol=1e-12, atol=1e-14)
    np.testing.assert_array_equal(out["weight"].data, expect_w)


def _random_obs(nants, ntimes, nchan, npol, seed, dtype=torch.complex128):
    from ska_sdp_func_python_amd import simulation
    rng = np.random.default_rng(seed)
    pf = {1: "stokesI", 2: "linearnp", 4: "linear"}[npol]
    vis = simulation.make_visibility("LOW", nants=nants, ntimes=ntimes, nchan=nchan, f_lo=1e8,
                                     f_hi=1.1e8, ha_span_h=0.5, polarisation_frame=pf, autos=True)
    shape = vis.vis.shape
    v = rng.normal(size=shape) + 1j * rng.normal(size=shape)
    m = rng.normal(size=shape) + 1j * rng.normal(size=shape)
    m[rng.uniform(size=shape) < 0.02] = 0.0
    w = rng.uniform(0.5, 2.0, shape)
    f = (rng.uniform(size=shape) < 0.05).astype(np.int64)
    return vis, v, m, w, f


@pytest.mark.parametrize("npol,nchan_g", [(1, 1), (4, 8), (2, 1)])
def test_point_sums_match_oracle(npol, nchan_g):
    """divide_visibility + per-gain-row sums in canonical baseline order, 64
    stations with autocorrelations, 12 times in 3 gain rows, 8 channels."""
    from ska_sdp_func_python_amd import kernels
    vis, v, m, w, f = _random_obs(64, 12, 8, npol, seed=npol)
    time = np.asarray(vis.time.data)
    gt_time = time[[1, 5, 9]]
    interval = np.full(3, 4.0 * float(np.median(np.diff(time))))
    xb_ref, xwt_ref = co.point_sums(v, w, f, time, gt_time, interval, nchan_g, model=m)
    bl = np.asarray(vis.baselines.data)
    perm, conj, _, _ = kernels.canonical_baselines(bl[:, 0], bl[:, 1], 64)
    ptr, idx = [0], []
    for r in range(3):
        sel = np.nonzero((time >= gt_time[r] - interval[r] / 2) & (time <= gt_time[r] + interval[r] / 2))[0]
        idx += sel.tolist()
        ptr.append(len(idx))
    d = lambda a, dt=None: torch.as_tensor(np.ascontiguousarray(a), device="cuda", dtype=dt)  # noqa: E731
    xb, xwt = kernels.point_sums(d(v), d(m), d(w), d(f), d(ptr, torch.int32), d(idx, torch.int32),
                                 nchan_g, perm=d(np.asarray(perm, np.int32)),
                                 conj=d(np.asarray(conj, np.uint8)))
    exp_xb = xb_ref[:, perm]
    exp_xb[:, conj] = np.conj(exp_xb[:, conj])
    np.testing.assert_allclose(xb.cpu().numpy(), exp_xb, rtol=1e-12, atol=1e-10)
    np.testing.assert_allclose(xwt.cpu().numpy(), xwt_ref[:, perm], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("dtype", [torch.complex128, torch.complex64])
def test_divide_visibility_matches_oracle(dtype):
    from ska_sdp_func_python_amd.visibility.operations import divide_visibility
    vis, v, m, w, f = _random_obs(16, 5, 3, 4, seed=7)
    vis["vis"] = torch.as_tensor(v, device="cuda").to(dtype)
    vis["weight"] = torch.as_tensor(w, device="cuda")
    vis["flags"] = torch.as_tensor(f, device="cuda")
    model = vis.copy(deep=True)
    model["vis"] = torch.as_tensor(m, device="cuda").to(dtype)
    out = divide_visibility(vis, model)
    vv = v.astype(np.complex64).astype(complex) if dtype == torch.complex64 else v
    mm = m.astype(np.complex64).astype(complex) if dtype == torch.complex64 else m
    keep = 1 - f
    xwt = np.abs(mm * keep) ** 2 * (w * keep)
    x = np.zeros_like(vv)
    x[xwt > 0] = (vv * keep)[xwt > 0] / (mm * keep)[xwt > 0]
    tol = 1e-12 if dtype == torch.complex128 else 1e-6
    np.testing.assert_allclose(out.vis.data.cpu().numpy(), x, rtol=tol, atol=tol)
    np.testing.assert_allclose(out.weight.data.cpu().numpy(), xwt, rtol=1e-12)
