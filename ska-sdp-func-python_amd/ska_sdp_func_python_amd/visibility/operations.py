"""divide_visibility (reference src/ska_sdp_func_python/visibility/operations.py:145-189).

x = V / M where |M|^2 w > 0 (else 0), weight' = |M|^2 w -- the point-source
equivalent visibility that solve_gaintable averages; flagged vis, model and
weight as the reference's visibility_acc.flagged_* give them.  One HIP
kernel (sdp_hip_divide_vis) with numpy's complex division.
"""

import numpy as np
import torch

from .. import _device, kernels
from ..datamodels import Visibility


def concatenate_visibility(vis_list, dim="time"):
    """Reference visibility/operations.py:38-72 for ``dim="time"`` (the only
    use on this path, sky_model drivers): time-dimension arrays joined,
    the rest taken from the first."""
    if not len(vis_list) > 0:
        raise ValueError("concatenate_visibility: vis_list is empty")
    if dim != "time":
        raise ValueError(f"concatenate_visibility: dim {dim} is not supported here")
    first = vis_list[0]
    rep = {}
    for k in ("vis", "uvw", "weight", "imaging_weight", "flags", "time", "integration_time"):
        if k not in first._vars:
            continue
        parts = [v._vars[k] for v in vis_list]
        if isinstance(parts[0], torch.Tensor):
            rep[k] = torch.cat([p if isinstance(p, torch.Tensor) else torch.as_tensor(p, device=parts[0].device)
                                for p in parts], dim=0)
        else:
            rep[k] = np.concatenate([np.asarray(p) for p in parts], axis=0)
    return first._copy_with(deep=True, replace=rep)


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
