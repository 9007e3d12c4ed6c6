"""Phase rotation of visibilities on the device.

Mirrors reference ``src/ska_sdp_func_python/visibility/base.py``:
``calculate_visibility_phasor`` (:27-45) ``exp(-2 pi i uvw_lambda . [l, m, n-1])``
and ``phaserotate_visibility`` (:60-125): multiply by the conjugate phasor
(``inverse=False``) or the phasor (``inverse=True``); returns a new
Visibility, or the input unchanged when |n-1| < 1e-15.  The phasor is formed
in fp64 on the GPU.
"""

import math

import torch

from .. import _device
from ..datamodels import C_M_S
from ..util.coordinate_support import skycoord_to_lmn, uvw_to_xyz, xyz_to_uvw


def _phase_turns(vis, direction):
    l, m, nm1 = skycoord_to_lmn(direction, vis.phasecentre)
    uvw = _device.to_dev(vis.uvw.data, torch.float64)
    freq = _device.to_dev(vis.frequency.data, torch.float64)
    s = torch.tensor([l, m, nm1], dtype=torch.float64, device=uvw.device)
    dot = (uvw * s).sum(-1)  # metres, [t, b]
    return dot[..., None] * (freq / C_M_S)  # turns, [t, b, f]


def calculate_visibility_phasor(direction, vis):
    """[t, b, f, p] complex128 phasor (device tensor)."""
    ph = _phase_turns(vis, direction)
    ph = ph - torch.round(ph)
    phasor = torch.polar(torch.ones_like(ph), -2.0 * math.pi * ph)
    npol = vis.vis.shape[-1]
    return phasor[..., None].expand(*phasor.shape, npol)


def phaserotate_visibility(vis, newphasecentre, tangent=True, inverse=False):
    _, _, n = skycoord_to_lmn(newphasecentre, vis.phasecentre)
    if abs(n) < 1e-15:
        return vis
    newvis = vis.copy(deep=True)
    ph = _phase_turns(vis, newphasecentre)
    ph = ph - torch.round(ph)
    # inverse=False multiplies by conj(phasor) = exp(+2 pi i phase)
    rot = torch.polar(torch.ones_like(ph), (2.0 * math.pi * ph) * (1.0 if not inverse else -1.0))
    v = _device.to_dev(newvis["vis"].data)
    v = v * rot[..., None].to(v.dtype)
    newvis["vis"].data = _device.like_input(v, vis["vis"].data)
    if not tangent:
        uvw = vis.uvw.data
        uvw_h = uvw.detach().cpu().numpy() if isinstance(uvw, torch.Tensor) else uvw
        nrows, nbl, _ = uvw_h.shape
        xyz = uvw_to_xyz(uvw_h.reshape(-1, 3), ha=-vis.phasecentre.ra.rad, dec=vis.phasecentre.dec.rad)
        new_uvw = xyz_to_uvw(xyz, ha=-newphasecentre.ra.rad, dec=newphasecentre.dec.rad)
        new_uvw = new_uvw.reshape(nrows, nbl, 3)
        newvis["uvw"].data = _device.like_input(_device.to_dev(new_uvw), uvw)
        newvis.attrs["phasecentre"] = newphasecentre
    return newvis
