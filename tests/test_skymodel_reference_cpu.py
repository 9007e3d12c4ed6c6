"""CPU: the oracle composition tests/test_gpu_skymodel.py checks the HIP
sky-model drivers against (ref_oracle.dft_cpu_looped + nufft_oracle exact
sums + calops_oracle.apply_gaintable, with the driver's mask / beam /
normalisation steps restated) equals the reference's own drivers executed
on the same case (tests/golden/skymodel.npz, make_golden.make_skymodel:
skymodel_imaging.py, imaging.py, ng.py, dft.py, apply_gaintable from the
reference sources, ducc0 as its exact sums) -- pinning the restatement."""

import numpy as np

import calops_oracle as co
import nufft_oracle as orc
from conftest import golden, rel_rms
from skymodel_case import _pb, _setup
from test_gpu_skymodel import FLIP_UW, _expected_predict


def test_restated_predict_matches_reference_execution():
    ref = golden("skymodel.npz")
    vis, sm, cell = _setup()
    g = sm.gaintable
    for use_pb in (False, True):
        beam = _pb(sm.image) if use_pb else None
        expect = _expected_predict(vis, sm, cell, beam)
        expect, _ = co.apply_gaintable(expect, np.asarray(vis.weight.data),
                                       np.asarray(vis.flags.data), np.asarray(vis.time.data),
                                       np.asarray(vis.baselines.data), g["gain"].data, g.time.data,
                                       g.interval.data, inverse=True)
        assert rel_rms(expect, ref[f"predict_pb{int(use_pb)}"]) < 1e-10


def test_restated_invert_matches_reference_execution():
    ref = golden("skymodel.npz")
    vis, sm, cell = _setup(seed=5)
    vis["vis"].data = ref["invert_vis"]
    g = sm.gaintable
    cal, _ = co.apply_gaintable(vis.vis.data, np.asarray(vis.weight.data), np.asarray(vis.flags.data),
                                np.asarray(vis.time.data), np.asarray(vis.baselines.data), g["gain"].data,
                                g.time.data, g.interval.data, inverse=False)
    f = np.asarray(vis.frequency.data)
    uvw = np.asarray(vis.uvw.data)
    npix = sm.image["pixels"].data.shape[-1]
    mask = sm.mask["pixels"].data[0, 0]
    d = orc.ms2dirty_exact(uvw.reshape(-1, 3) * FLIP_UW, f, cal.reshape(-1, len(f)), None, npix,
                           npix, cell, cell, True).T / cal[..., 0].size
    assert rel_rms(d * mask, ref["invert_pb0_dirty"][0, 0]) < 1e-10
    beam = _pb(sm.image)
    flat = mask * beam["pixels"].data[0, 0]
    sd = np.zeros((npix, npix))
    sf = np.zeros((npix, npix))
    for t in range(uvw.shape[0]):
        dt = orc.ms2dirty_exact(uvw[t] * FLIP_UW, f, cal[t].reshape(-1, len(f)), None, npix, npix,
                                cell, cell, True).T
        sd += flat * dt
        sf += flat * flat * cal[t][..., 0].size
    maxwt = sf.max()
    assert rel_rms(sd / maxwt, ref["invert_pb1_dirty"][0, 0]) < 1e-10
    np.testing.assert_allclose(np.sqrt(np.sqrt(sf / maxwt)), ref["invert_pb1_weights"][0, 0],
                               rtol=1e-12)


def test_restated_cube_matches_reference_execution():
    """The cube of the fixture (3 visibility channels onto 2 image channels,
    vis_to_im = [0, 0, 1]): each image channel is the exact sum over ITS
    visibility channels (the reference adds one ducc0 call per channel,
    ng.py:259-289; invert_ng now grids a run of them in one call), sumwt
    counts each channel once; predict puts image channel vis_to_im[c] on
    visibility channel c."""
    from skymodel_case import cube_case
    ref = golden("skymodel.npz")
    vis, sm, cell = _setup(seed=5)
    vis["vis"].data = ref["invert_vis"]
    _, px = cube_case(sm.image, vis)
    f = np.asarray(vis.frequency.data)
    uvw = np.asarray(vis.uvw.data).reshape(-1, 3) * FLIP_UW
    ms = np.asarray(vis.vis.data)[..., 0].reshape(-1, len(f))
    wt = np.asarray(vis.imaging_weight.data)[..., 0].reshape(-1, len(f))
    npix = px.shape[-1]
    for ichan, chans in ((0, [0, 1]), (1, [2])):
        d = orc.ms2dirty_exact(uvw, f[chans], ms[:, chans], wt[:, chans], npix, npix, cell, cell,
                               True).T
        sw = wt[:, chans].sum()
        assert abs(sw - ref["invert_cube_sumwt"][ichan, 0]) <= 1e-12 * sw
        assert rel_rms(d / sw, ref["invert_cube_dirty"][ichan, 0]) < 1e-10
    v = np.stack([orc.dirty2ms_exact(uvw, f[c:c + 1], px[ic, 0].T, None, cell, cell, True)[:, 0]
                  for c, ic in enumerate((0, 0, 1))], axis=1)
    assert rel_rms(v, ref["predict_cube_vis"][..., 0].reshape(-1, len(f))) < 1e-10
