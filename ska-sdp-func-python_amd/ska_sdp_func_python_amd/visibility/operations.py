"""divide_visibility (reference src/ska_sdp_func_python/visibility/operations.py:145-189).

x = V / M where |M|^2 w > 0 (else 0), weight' = |M|^2 w -- the point-source
equivalent visibility that solve_gaintable averages.  Computed on the device.
"""

import torch

from .. import _device
from ..datamodels import Visibility


def divide_visibility(vis, modelvis):
    v = _device.to_dev(vis.visibility_acc.flagged_vis).to(torch.complex128)
    m = _device.to_dev(modelvis.visibility_acc.flagged_vis).to(torch.complex128)
    w = _device.to_dev(vis.visibility_acc.flagged_weight).to(torch.float64)
    xwt = (m.abs() ** 2) * w
    mask = xwt > 0.0
    x = torch.where(mask, v / torch.where(mask, m, torch.ones_like(m)), torch.zeros_like(v))
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
