"""GPU parity of the sky-component DFT (sdp_hip_dft_point_*) against the
reference's dft_cpu_looped outputs (tests/golden/dft_*.npz).
Tolerance: complex128 output (fp64 sincos and sums, the reference's dtype)
|error| RMS / |vis| RMS < 1e-11; complex64 output (fp32 sincos) < 2e-6."""

import numpy as np
import pytest
import torch

from conftest import golden, rel_rms

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag", ["p4", "p1_bcast", "p2"])
def test_dft_point_v00_matches_reference(tag):
    from ska_sdp_func_python_amd.imaging.dft import dft_kernel
    g = golden(f"dft_{tag}.npz")
    for name in (None, "cpu_looped", "gpu_cupy_raw", "proc_func", "hip"):
        vis = dft_kernel(g["direction_cosines"], g["vfluxes"], g["uvw_lambda"], name)
        assert rel_rms(vis, g["vis"]) < 1e-11


def test_dft_unknown_kernel_raises():
    from ska_sdp_func_python_amd.imaging.dft import dft_kernel
    g = golden("dft_p4.npz")
    with pytest.raises(ValueError):
        dft_kernel(g["direction_cosines"], g["vfluxes"], g["uvw_lambda"], "nope")


def test_dft_skycomponent_qa_known_answers():
    """reference tests/imaging/test_dft_skycomponent_visibility_kernels.py:33-36."""
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd import simulation
    from ska_sdp_func_python_amd.imaging import dft_skycomponent_visibility
    pc = dm.SkyCoord(180.0, -35.0, unit="deg")
    freq = np.linspace(1.0e8, 1.1e8, 6)
    vis = simulation.make_visibility("LOW", nants=40, ntimes=2, nchan=6, f_lo=1.0e8, f_hi=1.1e8,
                                     polarisation_frame="linear", phasecentre=pc)
    comp = dm.SkyComponent(dm.SkyCoord(181.0, -35.0, unit="deg"), freq,
                           flux=np.array(6 * [100.0, 20.0, -10.0, 1.0]).reshape(6, 4),
                           polarisation_frame=dm.PolarisationFrame("stokesIQUV"))
    res = dft_skycomponent_visibility(vis, 20 * [comp])
    qa = res.visibility_acc.qa_visibility()
    np.testing.assert_almost_equal(qa.data["maxabs"], 2400.0, decimal=3)
    np.testing.assert_almost_equal(qa.data["minabs"], 200.9975124, decimal=3)
    np.testing.assert_almost_equal(qa.data["rms"], 942.9223125, decimal=3)


def test_dft_metres_matches_lambda_form_at_scale():
    """The fused-lambda entry point equals the uvw_lambda one (1e5 vis, 64 comps)."""
    from ska_sdp_func_python_amd import kernels
    rng = np.random.default_rng(1)
    dev = torch.device("cuda:0")
    nrow, nchan, ncomp = 20000, 5, 64
    freq = np.linspace(1e9, 1.4e9, nchan)
    uvw = rng.normal(0, 3e4, (nrow, 3))
    lm = rng.uniform(-0.02, 0.02, (ncomp, 2))
    dc = np.concatenate([lm, (np.sqrt(1 - (lm ** 2).sum(1)) - 1)[:, None]], 1)
    flux = rng.uniform(0.1, 2, (ncomp, 1, 1)).astype(complex)
    uvwl = uvw[:, None, :] * (freq / 299792458.0)[None, :, None]
    a = kernels.dft_point(torch.as_tensor(dc, device=dev), torch.as_tensor(flux, device=dev),
                          torch.as_tensor(uvw, device=dev), freq=torch.as_tensor(freq, device=dev))
    b = kernels.dft_point(torch.as_tensor(dc, device=dev), torch.as_tensor(flux, device=dev),
                          torch.as_tensor(uvwl, device=dev))
    assert rel_rms(a.cpu().numpy(), b.cpu().numpy()) < 1e-6
    # spot-check a few rows against fp64
    ph = np.exp(-2j * np.pi * np.einsum("rfs,cs->rfc", uvwl[:50], dc))
    ref = (ph * flux[:, 0, 0][None, None, :]).sum(-1)
    assert rel_rms(a.cpu().numpy()[:50, :, 0], ref) < 2e-6


def test_dft_c128_output_is_fp64_exact():
    """A complex128 output runs the phase's sincos, the flux and the sums in
    fp64 (the reference's numpy dtype): the direct fp64 sum to 1e-11 (the
    phase reaches 10^3 turns); the complex64 output keeps fp32 sincos
    (< 2e-6)."""
    from ska_sdp_func_python_amd import kernels
    rng = np.random.default_rng(2)
    dev = torch.device("cuda:0")
    nrow, nchan, ncomp = 3000, 3, 100
    freq = np.linspace(1e9, 1.4e9, nchan)
    uvw = rng.normal(0, 3e4, (nrow, 3))
    lm = rng.uniform(-0.02, 0.02, (ncomp, 2))
    dc = np.concatenate([lm, (np.sqrt(1 - (lm ** 2).sum(1)) - 1)[:, None]], 1)
    flux = (rng.uniform(0.1, 2, (ncomp, 1, 2)) + 1j * rng.uniform(-0.1, 0.1, (ncomp, 1, 2)))
    uvwl = uvw[:, None, :] * (freq / 299792458.0)[None, :, None]
    ph = np.exp(-2j * np.pi * np.einsum("rfs,cs->rfc", uvwl, dc))
    ref = np.einsum("rfc,cp->rfp", ph, flux[:, 0, :])
    args = (torch.as_tensor(dc, device=dev), torch.as_tensor(flux, device=dev),
            torch.as_tensor(uvw, device=dev))
    a = kernels.dft_point(*args, freq=torch.as_tensor(freq, device=dev),
                          vis_dtype=torch.complex128)
    b = kernels.dft_point(*args, freq=torch.as_tensor(freq, device=dev))
    assert rel_rms(a.cpu().numpy(), ref) < 1e-11
    assert rel_rms(b.cpu().numpy(), ref) < 2e-6
