"""Imaging helpers around the hot path (reference src/ska_sdp_func_python/imaging/base.py).

* ``shift_vis_to_image`` (:48-92): rotate to the image centre pixel
  (nx//2+1, ny//2+1, 1-based) when it differs from the vis phase centre.
* ``normalise_sumwt`` (:95-155): divide each [chan, pol] plane by sumwt, or
  zero it when sumwt <= 0 (2-D sumwt); the 4-D (image) form follows :129-149.
* ``predict_awprojection`` / ``invert_awprojection`` (:158-259) over the HIP
  convolution-function gridder (grid_data.gridding).
* ``fill_vis_for_psf`` (:262-296).
"""

import logging

import numpy as np
import torch

from .. import _device
from ..datamodels import (PolarisationFrame, create_griddata_from_image, pixel_to_skycoord)
from ..util.coordinate_support import skycoord_to_lmn
from ..visibility.base import phaserotate_visibility

log = logging.getLogger("func-python-logger")


def shift_vis_to_image(vis, im, tangent=True, inverse=False):
    ny = im["pixels"].data.shape[2]
    nx = im["pixels"].data.shape[3]
    image_phasecentre = pixel_to_skycoord(nx // 2 + 1, ny // 2 + 1, im.image_acc.wcs, origin=1)
    if vis.phasecentre.separation(image_phasecentre).rad > 1e-15:
        if inverse:
            log.debug("shift_vis_from_image: shifting phasecentre from image phase centre %s "
                      "to visibility phasecentre %s", image_phasecentre, vis.phasecentre)
        else:
            log.debug("shift_vis_from_image: shifting phasecentre from vis phasecentre %s to "
                      "image phasecentre %s", vis.phasecentre, image_phasecentre)
        vis = phaserotate_visibility(vis, image_phasecentre, tangent=tangent, inverse=inverse)
        vis.attrs["phasecentre"] = im.image_acc.phasecentre
    return vis


def shift_lmn(vis, im):
    """(l, m, n-1) by which ``shift_vis_to_image(vis, im, tangent=True)``
    would rotate the visibilities, or None when it would leave them alone
    (same two tests: phase-centre separation > 1e-15 rad, reference
    imaging/base.py:71-75, and |n-1| >= 1e-15, visibility/base.py:78-82).
    The fused NUFFT entry points apply that rotation on the fly."""
    ny = im["pixels"].data.shape[2]
    nx = im["pixels"].data.shape[3]
    image_phasecentre = pixel_to_skycoord(nx // 2 + 1, ny // 2 + 1, im.image_acc.wcs, origin=1)
    if vis.phasecentre.separation(image_phasecentre).rad <= 1e-15:
        return None
    l, m, n = skycoord_to_lmn(image_phasecentre, vis.phasecentre)
    if abs(n) < 1e-15:
        return None
    return l, m, n


def normalise_sumwt(im, sumwt, min_weight=0.1, flat_sky=False):
    pixels = im["pixels"].data
    nchan, npol = pixels.shape[0], pixels.shape[1]
    assert sumwt is not None
    if isinstance(sumwt, np.ndarray):
        assert nchan == sumwt.shape[0]
        assert npol == sumwt.shape[1]
        for chan in range(nchan):
            for pol in range(npol):
                if sumwt[chan, pol] > 0.0:
                    pixels[chan, pol] = pixels[chan, pol] / sumwt[chan, pol]
                else:
                    pixels[chan, pol] = 0.0
    elif tuple(pixels.shape) == tuple(sumwt["pixels"].data.shape):
        sw = sumwt["pixels"].data
        maxwt = float(sw.max())
        minwt = min_weight * maxwt
        cy, cx = sw.shape[2] // 2, sw.shape[3] // 2
        for chan in range(nchan):
            for pol in range(npol):
                if flat_sky:
                    norm = (sw[chan, pol, cy, cx] * sw[chan, pol]) ** 0.5
                    big = norm > minwt
                    pixels[chan, pol][big] /= norm[big]
                    pixels[chan, pol][~big] /= maxwt
                else:
                    pixels[chan, pol] /= maxwt
                    sw[chan, pol] /= maxwt
                    sumwt["pixels"].data = sw ** 0.5
    else:
        raise ValueError("sumwt is not a 2D or 4D array - cannot perform normalisation")
    im["pixels"].data = pixels
    return im


def fill_vis_for_psf(svis):
    pf = svis.visibility_acc.polarisation_frame
    v = svis["vis"].data
    if pf in (PolarisationFrame("linear"), PolarisationFrame("circular")):
        v[..., 0] = 1.0 + 0.0j
        v[..., 1:3] = 0.0 + 0.0j
        v[..., 3] = 1.0 + 0.0j
    elif pf in (PolarisationFrame("linearnp"), PolarisationFrame("circularnp"),
                PolarisationFrame("stokesI")):
        v[...] = 1.0 + 0.0j
    else:
        raise ValueError(f"Cannot calculate PSF for {pf}")
    return svis


def predict_awprojection(vis, model, gcfcf=None):
    from ..grid_data.gridding import degrid_visibility_from_griddata, fft_image_to_griddata
    from ..image_operations import convert_stokes_to_polimage

    if model is None:
        return vis
    assert not np.isnan(float(np.sum(np.asarray(_host(model["pixels"].data))))), \
        "NaNs present in input model"
    if gcfcf is None:
        raise ValueError("predict_awprojection: gcfcf not specified")
    gcf, cf = gcfcf(model)
    griddata = create_griddata_from_image(model, polarisation_frame=vis.visibility_acc.polarisation_frame)
    polmodel = convert_stokes_to_polimage(model, vis.visibility_acc.polarisation_frame)
    griddata = fft_image_to_griddata(polmodel, griddata, gcf)
    vis = degrid_visibility_from_griddata(vis, griddata=griddata, cf=cf)
    return shift_vis_to_image(vis, model, tangent=True, inverse=True)


def invert_awprojection(vis, im, dopsf=False, normalise=True, gcfcf=None):
    from ..grid_data.gridding import fft_griddata_to_image, grid_visibility_to_griddata
    from ..image_operations import convert_polimage_to_stokes

    svis = vis.copy(deep=True)
    if dopsf:
        svis = fill_vis_for_psf(svis)
    svis = shift_vis_to_image(svis, im, tangent=True, inverse=False)
    griddata = create_griddata_from_image(im, polarisation_frame=vis.visibility_acc.polarisation_frame)
    if gcfcf is None:
        raise ValueError("invert_awprojection: gcfcf not specified")
    gcf, cf = gcfcf(im)
    griddata, sumwt = grid_visibility_to_griddata(svis, griddata=griddata, cf=cf)
    result = fft_griddata_to_image(griddata, im, gcf)
    if normalise:
        result = normalise_sumwt(result, sumwt)
    result = convert_polimage_to_stokes(result)
    assert not np.isnan(float(np.sum(np.asarray(_host(result["pixels"].data))))), \
        "NaNs present in output image"
    return result, sumwt


def _host(a):
    return a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
