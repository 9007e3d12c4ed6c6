"""Imaging weights on MI355X: weight_visibility and the two tapers.

Mirrors reference ``src/ska_sdp_func_python/imaging/weighting.py``:

* ``weight_visibility`` (:35-68): natural -> copy of the weight; uniform /
  robust -> grid the flagged weights on the model's uv grid
  (``grid_visibility_weight_to_griddata``) and reweight
  (``griddata_visibility_reweight``).  Here the weight grid stays on the
  device between the two HIP kernels.
* ``taper_visibility_gaussian`` (:71-101) and ``taper_visibility_tukey``
  (:104-136): imaging_weight = flagged imaging weight * taper(|uv|), in the
  sdp_hip_taper kernel.
"""

import numpy as np
import torch

from .. import _device, kernels
from ..datamodels import Image, create_griddata_from_image
from ..grid_data import gridding as _gd


def weight_visibility(vis, model, weighting="uniform", robustness=0.0):
    assert isinstance(model, Image), model
    assert model.image_acc.is_canonical()
    if weighting == "natural":
        return _gd.griddata_visibility_reweight(vis, None, weighting=weighting)
    griddata = create_griddata_from_image(model,
                                          polarisation_frame=vis.visibility_acc.polarisation_frame)
    grid, sumwt = _gd.grid_weights_device(vis, griddata)
    dev = grid.device
    v2i = torch.as_tensor(_gd._vis_to_im(griddata, vis.frequency.data), dtype=torch.int32,
                          device=dev)
    return _gd._reweight_device(vis, grid, _gd._uv_wcs(griddata), v2i, weighting, robustness,
                                sumwt)


def _taper(vis, kind, param):
    dev = _device.device()
    nrows, nbaselines, nvchan, nvpol = vis.vis.shape
    uvw, freq, _, fl = _gd._weight_inputs(vis, dev)
    iw = _device.to_dev(vis.imaging_weight.data, torch.float64, dev).reshape(
        nrows * nbaselines, nvchan, nvpol).contiguous()
    kernels.taper(uvw, freq, fl, iw, kind, param)
    _gd._store(vis, "imaging_weight", iw)
    return vis


def taper_visibility_gaussian(vis, beam=None):
    """Reference weighting.py:71-101 (beam = FWHM in radians)."""
    if beam is None:
        raise ValueError("Beam size not specified for Gaussian taper")
    scale_factor = np.pi ** 2 * beam ** 2 / (4.0 * np.log(2.0))
    return _taper(vis, "gaussian", scale_factor)


def taper_visibility_tukey(vis, tukey=0.1):
    """Reference weighting.py:104-136 (WSClean's tukey taper of |uv| / max|uv|)."""
    return _taper(vis, "tukey", tukey)
