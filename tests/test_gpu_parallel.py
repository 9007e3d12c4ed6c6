"""GPU: the sharding helpers of parallel.py drive the real HIP kernels
(single rank, no process group: the local compute path of every shard)."""

import numpy as np
import pytest
import torch

import nufft_oracle as orc
import ref_oracle as ro
from conftest import rel_rms

pytestmark = pytest.mark.gpu
FLIP = np.array([-1.0, 1.0, -1.0])


def T(a):
    return torch.as_tensor(np.asarray(a), device=torch.device("cuda:0"))


def test_invert_and_predict_sharded_match_exact():
    from ska_sdp_func_python_amd import parallel
    rng = np.random.default_rng(21)
    nrow, nchan, npix = 300, 3, 64
    freq = np.linspace(1.0e9, 1.2e9, nchan)
    uvw = rng.uniform(-1, 1, (nrow, 3)) * 1500 * orc.C_LIGHT / freq.max()
    vis = rng.normal(size=(nrow, nchan)) + 1j * rng.normal(size=(nrow, nchan))
    wgt = rng.uniform(0.5, 1.5, (nrow, nchan)).astype(np.float32)
    cell = 0.45 / 1500
    img, sw = parallel.invert_sharded(T(uvw), T(freq), T(vis).to(torch.complex64), T(wgt), npix, cell,
                                      1e-7, True)
    ex = orc.ms2dirty_exact(uvw * FLIP, freq, vis, wgt, npix, npix, cell, cell, True).T / wgt.sum()
    assert rel_rms(img.cpu().numpy(), ex) < 5e-6
    model = rng.normal(size=(npix, npix))  # [y, x]
    v = parallel.predict_sharded(T(uvw), T(freq), T(model), cell, 1e-7, True,
                                 vis_dtype=torch.complex128)
    exv = orc.dirty2ms_exact(uvw * FLIP, freq, model.T, None, cell, cell, True)
    assert rel_rms(v.cpu().numpy(), exv) < 5e-6


def test_dft_sharded_matches_oracle():
    from ska_sdp_func_python_amd import parallel
    rng = np.random.default_rng(22)
    uvw = rng.normal(0, 3000, (500, 3))
    freq = np.array([1.0e9, 1.3e9])
    lm = rng.uniform(-0.03, 0.03, (7, 2))
    dc = np.concatenate([lm, (np.sqrt(1 - (lm ** 2).sum(1)) - 1)[:, None]], 1)
    fl = rng.uniform(0.5, 2, (7, 1, 1)) + 0j
    v = parallel.dft_sharded(T(dc), T(fl), T(uvw), freq=T(freq))
    ref = ro.dft_cpu_looped(dc, uvw[:, None, :] * (freq / 299792458.0)[None, :, None], fl)
    assert rel_rms(v.cpu().numpy(), ref) < 2e-6


@pytest.mark.parametrize("norm", ["mean", "median"])
def test_solve_gains_sharded_normalises(norm):
    from ska_sdp_func_python_amd import kernels, parallel
    rng = np.random.default_rng(23)
    nants, nrows, nchan = 12, 3, 2
    a1, a2 = np.triu_indices(nants, 1)
    g = rng.lognormal(0, 0.2, (nrows, nants, nchan)) * np.exp(1j * rng.normal(0, 0.3, (nrows, nants, nchan)))
    xb = (g[:, a1] * np.conj(g[:, a2]))[..., None]
    perm, conj, rs, ant2 = kernels.canonical_baselines(a1, a2, nants)
    gain = torch.ones((nrows, nants, nchan, 1, 1), dtype=torch.complex128, device="cuda:0")
    gwt = torch.zeros((nrows, nants, nchan, 1, 1), dtype=torch.float64, device="cuda:0")
    parallel.solve_gains_sharded(T(xb[:, perm]), T(np.ones(xb.shape)), gain, gwt, rs, ant2, 0,
                                 phase_only=False, normalise_gains=norm)
    ga = gain.abs().cpu().numpy()
    stat = np.median(ga) if norm == "median" else np.mean(ga)
    assert abs(stat - 1.0) < 1e-12
    # solutions reproduce the data up to the (global) normalisation scale
    gs = gain.cpu().numpy()[..., 0, 0]
    model = gs[:, a1] * np.conj(gs[:, a2])
    ratio = (xb[..., 0] / model).real
    assert np.allclose(ratio, ratio.flat[0], rtol=1e-5)
