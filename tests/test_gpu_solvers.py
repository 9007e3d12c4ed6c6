"""GPU parity of solve_gaintable (batched StefCal, sdp_hip_solve_gains)
against the reference's own solve_gaintable run on the same inputs
(tests/golden/solve_*.npz).

The kernel stores the normalised point-source vis / weights in fp32 and
iterates in fp64.  A relative perturbation of 6e-8 in x moves the fixed point
of the substitution g_j = sum_i g_i x_ij w_ij / sum_i |g_i|^2 w_ij by the same
relative order, far below the reference's stopping tolerance tol = 1e-6, so
the stopping iteration and the gains agree: measured max |dgain| 4.5e-8 over
the seven fixtures, 6e-9 on 512-station C5 rows with equal iteration counts
(scripts/gpu_stefcal_parity.py, tests/test_gpu_fullsize.py).  Asserted:
gains to 1e-6 absolute (= tol), weights to 1e-6 relative, residuals to 1e-7."""

import numpy as np
import pytest

from conftest import golden
from gpu_helpers import vis_from_arrays

pytestmark = pytest.mark.gpu

CASES = ["scalar_T_phase", "scalar_B_amp_mean", "scalar_T_amp_median", "matrix_crosspol_B",
         "nocross_linear_T", "nocross_linearnp_B", "nocross_circular_T"]


def _tables(g):
    from ska_sdp_func_python_amd import datamodels as dm
    pf = str(g["pol_frame"])
    vis = vis_from_arrays(g["uvw"], g["frequency"], g["vis"], baselines=g["baselines"], pf=pf,
                          times=g["time"], integration_time=g["integration_time"])
    model = vis.copy(deep=True)
    model["vis"].data = g["model"].copy()
    gt = dm.create_gaintable_from_visibility(vis, jones_type=str(g["jones"]))
    gt["gain"].data = g["gain_in"].copy()
    gt["weight"].data = g["weight_in"].copy()
    return vis, model, gt


@pytest.mark.parametrize("case", CASES)
def test_solve_gaintable_matches_reference(case):
    from ska_sdp_func_python_amd.calibration import solve_gaintable
    g = golden(f"solve_{case}.npz")
    vis, model, gt = _tables(g)
    norm = str(g["normalise"])
    out = solve_gaintable(vis, model, gain_table=gt, phase_only=bool(g["phase_only"]),
                          niter=int(g["niter"]), tol=float(g["tol"]), crosspol=bool(g["crosspol"]),
                          normalise_gains=None if norm == "None" else norm, jones_type=str(g["jones"]))
    np.testing.assert_allclose(out["gain"].data, g["gain"], atol=1e-6)
    np.testing.assert_allclose(out["weight"].data, g["weight"], rtol=1e-6, atol=1e-12)
    np.testing.assert_allclose(out["residual"].data, g["residual"], rtol=1e-5, atol=1e-7)


def test_zero_model_raises():
    from ska_sdp_func_python_amd.calibration import solve_gaintable
    g = golden("solve_scalar_T_phase.npz")
    vis, model, gt = _tables(g)
    model["vis"].data[...] = 0.0
    with pytest.raises(ValueError):
        solve_gaintable(vis, model)


def test_recovers_simulated_gains_large():
    """512 antennas, 4 channels jointly: the solved phases match the truth up
    to the refant rotation (residual bound, cf. reference
    tests/calibration/test_chain_calibration.py:126-127)."""
    import torch
    from ska_sdp_func_python_amd import kernels
    rng = np.random.default_rng(1805550721)
    nants, nchan = 512, 4
    a1, a2 = np.triu_indices(nants, 1)
    g = np.exp(1j * rng.normal(0, 0.5, (nants, nchan)))
    xb = (g[a1] * np.conj(g[a2]))[None, :, :, None]
    wb = np.ones_like(xb.real)
    perm, conj, rs, ant2 = kernels.canonical_baselines(a1, a2, nants)
    dev = torch.device("cuda:0")
    gain = torch.ones((1, nants, nchan, 1, 1), dtype=torch.complex128, device=dev)
    gwt = torch.zeros((1, nants, nchan, 1, 1), dtype=torch.float64, device=dev)
    res, used = kernels.solve_gains(torch.as_tensor(xb[:, perm], device=dev),
                                    torch.as_tensor(wb[:, perm], device=dev), gain, gwt, rs, ant2,
                                    mode=0, niter=200, tol=1e-8, phase_only=True)
    sol = gain.cpu().numpy()[0, :, :, 0, 0]
    truth = g * np.exp(-1j * np.angle(g[0]))[None, :]
    assert np.max(np.abs(sol - truth)) < 1e-5
    assert float(res.max()) < 1.3e-6
    assert int(used[0]) <= 200


@pytest.mark.parametrize("nants", [37, 300])
def test_irregular_baselines_match_oracle(nants):
    """A sparse, ragged baseline set (60 % of the pairs, one antenna with no
    baselines at all, so CSR rows of every length and empty rows) with noisy
    data and random weights, two gain rows: the device solve against the
    restated reference solver (oracle/ref_oracle.stefcal_row) iteration for
    iteration (fixed niter, no early stop)."""
    import torch
    import ref_oracle as ro
    from ska_sdp_func_python_amd import kernels
    rng = np.random.default_rng(nants)
    nchan = 3
    a1, a2 = np.triu_indices(nants, 1)
    keep = (rng.uniform(size=a1.size) < 0.6) & (a1 != 7) & (a2 != 7)
    a1, a2 = a1[keep], a2[keep]
    g = np.exp(1j * rng.normal(0, 0.5, (nants, nchan))) * rng.uniform(0.8, 1.2, (nants, nchan))
    nsolve = 2
    xb = np.stack([(g[a1] * np.conj(g[a2])) * (1 + 0.05 * s) for s in range(nsolve)])[..., None]
    xb = xb + 0.02 * (rng.normal(size=xb.shape) + 1j * rng.normal(size=xb.shape))
    wb = rng.uniform(0.5, 2.0, xb.shape)
    perm, conj, rs, ant2 = kernels.canonical_baselines(a1, a2, nants)
    assert not np.any(conj)
    dev = torch.device("cuda:0")
    gain = torch.ones((nsolve, nants, nchan, 1, 1), dtype=torch.complex128, device=dev)
    gwt = torch.zeros((nsolve, nants, nchan, 1, 1), dtype=torch.float64, device=dev)
    res, used = kernels.solve_gains(torch.as_tensor(xb[:, perm], device=dev),
                                    torch.as_tensor(wb[:, perm], device=dev), gain, gwt, rs, ant2,
                                    mode=0, niter=12, tol=0.0, phase_only=False)
    bl = list(zip(a1, a2))
    for s in range(nsolve):
        eg, ew, er, eu = ro.stefcal_row(xb[s], wb[s], bl, nants,
                                        np.ones((nants, nchan, 1, 1), complex),
                                        np.zeros((nants, nchan, 1, 1)), niter=12, tol=0.0,
                                        phase_only=False)
        assert int(used[s]) == eu
        np.testing.assert_allclose(gain[s].cpu().numpy(), eg, atol=1e-6)
        np.testing.assert_allclose(gwt[s].cpu().numpy(), ew, rtol=1e-6, atol=1e-12)
        np.testing.assert_allclose(res[s].cpu().numpy(), er, rtol=1e-5, atol=1e-7)
