"""divide_visibility (reference src/ska_sdp_func_python/visibility/operations.py:145-189).

x = V / M where |M|^2 w > 0 (else 0), weight' = |M|^2 w -- the point-source
equivalent visibility that solve_gaintable averages; flagged vis, model and
weight as the reference's visibility_acc.flagged_* give them.  One HIP
kernel (sdp_hip_divide_vis) with numpy's complex division.
"""

import torch

from .. import _device, kernels
from ..datamodels import Visibility


def divide_visibility(vis, modelvis):
    dev = _device.device()
    v = _device.to_dev(vis["vis"].data, None, dev)
    if v.dtype not in (torch.complex64, torch.complex128):
        v = v.to(torch.complex128)
    v = v.contiguous()
    m = _device.to_dev(modelvis["vis"].data, v.dtype, dev).contiguous()
    w = _device.to_dev(vis["weight"].data, torch.float64, dev).contiguous()
    fl = _device.to_dev(vis["flags"].data, None, dev)
    if fl.dtype not in kernels._FLAG_DT:
        fl = fl.to(torch.int64)
    mfl = None
    if modelvis["flags"].data is not vis["flags"].data:
        mfl = _device.to_dev(modelvis["flags"].data, fl.dtype, dev)
    x, xwt = kernels.divide_vis(v, m, w, fl.contiguous(), model_flags=mfl)
    ref = vis["vis"].data
    out = Visibility.constructor(
        flags=vis.flags.data, baselines=vis.baselines.data, frequency=vis.frequency.data,
        channel_bandwidth=vis.channel_bandwidth.data, phasecentre=vis.phasecentre,
        configuration=vis.configuration, uvw=vis.uvw.data, time=vis.time.data,
        integration_time=vis.integration_time.data, vis=_device.like_input(x, ref),
        weight=_device.like_input(xwt, ref), source=vis.attrs.get("source"),
        meta=vis.attrs.get("meta"), polarisation_frame=vis.visibility_acc.polarisation_frame)
    out["imaging_weight"] = vis.imaging_weight.data
    return out
