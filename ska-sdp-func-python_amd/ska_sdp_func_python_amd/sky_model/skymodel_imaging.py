"""skymodel_predict_calibrate / skymodel_calibrate_invert on MI355X
(reference src/ska_sdp_func_python/sky_model/skymodel_imaging.py:23-235).

Drivers over the hot path: the components through the HIP DFT
(dft_skycomponent_visibility), the image through predict_ng / invert_ng (HIP
w-stacking NUFFT), the gain table through apply_gaintable (HIP), with the
reference's optional mask, per-time primary beam (``get_pb``) and
normalisation by the summed flat.  ``groupby("time")`` becomes one
Visibility view per time sample (datamodels.visibility_time_slices).
"""

import numpy as np

from ..calibration.operations import apply_gaintable
from ..datamodels import visibility_time_slices
from ..imaging.base import normalise_sumwt
from ..imaging.dft import dft_skycomponent_visibility
from ..imaging.imaging import invert_visibility, predict_visibility
from ..sky_component.operations import apply_beam_to_skycomponent
from ..visibility.operations import concatenate_visibility


def _np(a):
    return a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)


def _like(value, ref):
    """``value`` (numpy) on the side of ``ref`` (numpy or device tensor)."""
    if hasattr(ref, "detach"):
        import torch
        return torch.as_tensor(value, device=ref.device, dtype=ref.dtype)
    return value


def _dft_sky_component(vis_slice, skymodel, pb=None, dft_compute_kernel=None):
    """Reference skymodel_imaging.py:23-44."""
    comps = skymodel.components
    if skymodel.mask is not None or pb is not None:
        comps = [c.copy() for c in comps]
        if skymodel.mask is not None:
            comps = apply_beam_to_skycomponent(comps, skymodel.mask)
        if pb is not None:
            comps = apply_beam_to_skycomponent(comps, pb)
    return dft_skycomponent_visibility(vis_slice, comps, dft_compute_kernel=dft_compute_kernel)


def _fft_image(vis_slice, context, skymodel, pb=None, **kwargs):
    """Reference skymodel_imaging.py:47-66: predict the (masked, beamed)
    image and add it to the slice's visibilities."""
    imgv = vis_slice.copy(deep=True, zero=True)
    model = skymodel.image
    if skymodel.mask is not None or pb is not None:
        model = skymodel.image.copy(deep=True)
        px = _np(model["pixels"].data).copy()
        if skymodel.mask is not None:
            px = px * _np(skymodel.mask["pixels"].data)
        if pb is not None:
            px = px * _np(pb["pixels"].data)
        model["pixels"].data = _like(px, model["pixels"].data)
    imgv = predict_visibility(imgv, model, context=context, **kwargs)
    vis_slice["vis"].data += imgv["vis"].data


def _image_nonzero(skymodel):
    return skymodel.image is not None and np.max(np.abs(_np(skymodel.image["pixels"].data))) > 0.0


def skymodel_predict_calibrate(bvis, skymodel, context="ng", docal=False, inverse=True,
                               get_pb=None, **kwargs):
    v = bvis.copy(deep=True, zero=True)
    kernel = kwargs.get("dft_compute_kernel", None)
    if get_pb is not None:
        vis_slices = []
        for vis_slice in visibility_time_slices(v):
            pb = get_pb(vis_slice, skymodel.image)
            if len(skymodel.components) > 0:
                vis_slice = _dft_sky_component(vis_slice, skymodel, pb=pb, dft_compute_kernel=kernel)
            if _image_nonzero(skymodel):
                _fft_image(vis_slice, context, skymodel, pb=pb, **kwargs)
            vis_slices.append(vis_slice)
        v = concatenate_visibility(vis_slices, "time")
        if docal and skymodel.gaintable is not None:
            v = apply_gaintable(v, skymodel.gaintable, inverse=inverse)
        return v
    v = _dft_sky_component(v, skymodel, pb=None, dft_compute_kernel=kernel)
    if _image_nonzero(skymodel):
        _fft_image(v, context, skymodel, pb=None, **kwargs)
    if docal and skymodel.gaintable is not None:
        v = apply_gaintable(v, skymodel.gaintable, inverse=inverse)
    return v


def skymodel_calibrate_invert(bvis, skymodel, context="ng", docal=False, get_pb=None,
                              normalise=True, flat_sky=False, **kwargs):
    if skymodel.image is None:
        raise ValueError("skymodel image is None")
    bvis_cal = bvis.copy(deep=True)
    if docal and skymodel.gaintable is not None:
        bvis_cal = apply_gaintable(bvis_cal, skymodel.gaintable)
    if get_pb is not None:
        shape = skymodel.image["pixels"].data.shape
        sum_flats = np.zeros(shape)
        sum_dirtys = np.zeros(shape)
        for vis_slice in visibility_time_slices(bvis_cal):
            pb = get_pb(vis_slice, skymodel.image)
            dirty, sumwt = invert_visibility(vis_slice, skymodel.image, context=context,
                                             normalise=False, **kwargs)
            d = _np(dirty["pixels"].data)
            flat = np.ones_like(d)
            if skymodel.mask is not None:
                flat *= _np(skymodel.mask["pixels"].data)
            if pb is not None:
                flat *= _np(pb["pixels"].data)
            sum_dirtys += flat * d
            sum_flats += flat * flat * np.asarray(sumwt)[:, :, np.newaxis, np.newaxis]
        dirtys = skymodel.image.copy(deep=True)
        dirtys["pixels"].data = sum_dirtys
        flats = skymodel.image.copy(deep=True)
        flats["pixels"].data = sum_flats
        if normalise:
            dirtys = normalise_sumwt(dirtys, flats, flat_sky=flat_sky)
            flats["pixels"].data = np.sqrt(flats["pixels"].data)
        return dirtys, flats
    result = invert_visibility(bvis_cal, skymodel.image, context=context, **kwargs)
    if skymodel.mask is not None:
        px = result[0]["pixels"].data
        result[0]["pixels"].data = px * _like(_np(skymodel.mask["pixels"].data), px)
    return result
