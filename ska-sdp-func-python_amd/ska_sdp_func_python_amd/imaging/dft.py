"""Sky-component DFT predict on MI355X.

Mirrors reference ``src/ska_sdp_func_python/imaging/dft.py``:
``dft_skycomponent_visibility`` (:32-56, replaces ``vis["vis"]``),
``extract_direction_and_flux`` (:59-118: pol-frame conversion, cubic
frequency interpolation, lmn with n-1) and ``dft_kernel`` (:121-182).

Every ``dft_compute_kernel`` the reference knows ("cpu_looped",
"gpu_cupy_raw", "proc_func") and "hip" run the same HIP kernel
(sdp_hip_dft_point_*); unknown names raise ValueError like the reference.
Unlike the reference (Appendix B.1), no ska_sdp_func import is required.
"""

import collections.abc
import logging

import numpy as np
import torch
from scipy import interpolate

from .. import _device, kernels
from ..datamodels import convert_pol_frame
from ..util.coordinate_support import skycoord_to_lmn

log = logging.getLogger("func-python-logger")

KNOWN_KERNELS = ("cpu_looped", "gpu_cupy_raw", "proc_func", "hip")


def dft_skycomponent_visibility(vis, sc, dft_compute_kernel=None):
    if sc is None or (isinstance(sc, list) and len(sc) == 0):
        return vis
    _check_kernel(dft_compute_kernel)
    direction_cosines, vfluxes = extract_direction_and_flux(sc, vis)
    dev = _device.device()
    nt, nb, nchan, npol = vis.vis.shape
    uvw = _device.to_dev(vis.uvw.data, torch.float64, dev).reshape(nt * nb, 3)
    freq = _device.to_dev(np.asarray(vis.frequency.data, float), torch.float64, dev)
    ref = vis["vis"].data
    dtype = ref.dtype if isinstance(ref, torch.Tensor) else torch.complex128
    out = kernels.dft_point(_device.to_dev(direction_cosines, torch.float64, dev),
                            _device.to_dev(vfluxes, torch.complex128, dev), uvw, freq=freq,
                            vis_dtype=dtype if dtype in (torch.complex64, torch.complex128)
                            else torch.complex128)
    vis["vis"].data = _device.like_input(out.reshape(nt, nb, nchan, npol), ref)
    return vis


def extract_direction_and_flux(sc, vis):
    if not isinstance(sc, collections.abc.Iterable):
        sc = [sc]
    vfluxes = []
    direction_cosines = []
    vfreq = np.asarray(vis.frequency.data, float)
    for comp in sc:
        flux = comp.flux
        if comp.polarisation_frame != vis.visibility_acc.polarisation_frame:
            flux = convert_pol_frame(flux, comp.polarisation_frame,
                                     vis.visibility_acc.polarisation_frame)
        if len(comp.frequency) == len(vfreq) and np.allclose(comp.frequency, vfreq, rtol=1e-15):
            vflux = flux
        else:
            nchan, npol = flux.shape
            vflux = np.zeros([len(vfreq), npol], dtype=np.asarray(flux).dtype)
            if nchan > 1:
                for pol in range(flux.shape[1]):
                    fint = interpolate.interp1d(comp.frequency, comp.flux[:, pol], kind="cubic")
                    vflux[:, pol] = fint(vfreq)
            else:
                vflux = flux
        vfluxes.append(vflux)
        l, m, _ = skycoord_to_lmn(comp.direction, vis.phasecentre)
        direction_cosines.append(np.array([l, m, np.sqrt(1 - l ** 2 - m ** 2) - 1.0]))
    return np.array(direction_cosines), np.array(vfluxes).astype("complex")


def _check_kernel(name):
    if name is not None and name not in KNOWN_KERNELS:
        raise ValueError(f"dft_compute_kernel {name} not known")


def dft_kernel(direction_cosines, vfluxes, uvw_lambda, dft_compute_kernel=None):
    """vis [t, b, f, p] from uvw_lambda [t, b, f, 3] (reference dft.py:121)."""
    _check_kernel(dft_compute_kernel)
    dev = _device.device()
    uvwl = _device.to_dev(uvw_lambda, torch.float64, dev)
    nt, nb, nchan, _ = uvwl.shape
    fl = _device.to_dev(np.asarray(vfluxes), torch.complex128, dev)
    out = kernels.dft_point(_device.to_dev(direction_cosines, torch.float64, dev), fl,
                            uvwl.reshape(nt * nb, nchan, 3), vis_dtype=torch.complex128)
    return _device.like_input(out.reshape(nt, nb, nchan, -1), uvw_lambda)
