"""Stokes <-> polarisation image conversion used by the AW-projection wrappers
(reference src/ska_sdp_func_python/image/operations.py:78-170)."""

import numpy as np
import torch

from .datamodels import Image, PolarisationFrame, convert_pol_frame

_STOKES_FOR = {"linear": "stokesIQUV", "circular": "stokesIQUV", "linearnp": "stokesIQ",
               "circularnp": "stokesIV", "stokesI": "stokesI"}


def convert_stokes_to_polimage(im, polarisation_frame):
    if polarisation_frame.type not in _STOKES_FOR:
        raise ValueError(f"Cannot convert stokes to {polarisation_frame.type}")
    data = im["pixels"].data
    data = data.to(torch.complex128) if isinstance(data, torch.Tensor) else np.asarray(data).astype(complex)
    src = im.image_acc.polarisation_frame
    if polarisation_frame.type != "stokesI":
        data = convert_pol_frame(data, PolarisationFrame(_STOKES_FOR[polarisation_frame.type])
                                 if src.type != _STOKES_FOR[polarisation_frame.type] else src,
                                 polarisation_frame, polaxis=1)
    return Image.constructor(data=data, polarisation_frame=polarisation_frame,
                             wcs=im.image_acc.wcs)


def convert_polimage_to_stokes(im, complex_image=False):
    pf = im.image_acc.polarisation_frame
    data = im["pixels"].data
    if pf.type not in _STOKES_FOR:
        raise ValueError(f"Cannot convert {pf.type} to stokes")
    out_pf = PolarisationFrame(_STOKES_FOR[pf.type])
    if pf.type != "stokesI":
        data = convert_pol_frame(data, pf, out_pf, polaxis=1)
    if not complex_image:
        data = data.real
    return Image.constructor(data=data, polarisation_frame=out_pf, wcs=im.image_acc.wcs)
