"""apply_gaintable on MI355X (reference
``src/ska_sdp_func_python/calibration/operations.py:23-256``).

The reference's per gain row x vis row x baseline x channel Python loop
becomes one HIP kernel over (time, baseline, channel) (sdp_hip_apply_gains)
plus a small kernel forming the effective gains (the scalar reciprocal or
the 2x2 inverse with the singular-gain test).  The vis rows a gain row owns
are ``|t - T_r| < interval_r / 2`` (strict, operations.py:57-61).  When a
vis time falls in more than one gain row's window the reference applies
the rows one after another; so does this, one launch per gain row.  The
input Visibility is modified in place and returned, as in the reference.
"""

import logging

import numpy as np
import torch

from .. import _device, kernels

log = logging.getLogger("func-python-logger")


def _time_rows(vis_time, gt_time, interval):
    """[nrow_g][vis time indices] with the reference's strict window."""
    return [np.nonzero(np.abs(vis_time - gt_time[r]) < interval[r] / 2.0)[0]
            for r in range(len(gt_time))]


def _store(vis, name, value):
    cur = vis[name].data
    if _device.is_device(cur):
        if cur.data_ptr() != value.data_ptr():
            cur.copy_(value.reshape(cur.shape))
    else:
        cur[...] = value.reshape(cur.shape).cpu().numpy()


def apply_gaintable(vis, gt, inverse=False, use_flags=False):
    ntimes, nants, nchan, _, _ = gt.gain.shape
    if inverse:
        log.debug("apply_gaintable: Apply inverse gaintable")
    else:
        log.debug("apply_gaintable: Apply gaintable")
    if vis.visibility_acc.npol == 1:
        log.debug("apply_gaintable: scalar gains")
    dev = _device.device()
    vis_time = np.asarray(vis.time.data, dtype=float)
    rows = _time_rows(vis_time, np.asarray(gt.time.data, dtype=float),
                      np.asarray(gt.interval.data, dtype=float))
    nvt = len(vis_time)
    hits = np.zeros(nvt, dtype=int)
    for r in rows:
        hits[r] += 1
    if np.any(hits > 1):
        passes = [[r] for r in range(len(rows)) if len(rows[r])]  # sequential, as the reference
    else:
        passes = [list(range(len(rows)))]
    v = _device.to_dev(vis["vis"].data, None, dev)
    if v.dtype not in (torch.complex64, torch.complex128):
        v = v.to(torch.complex128)
    v = v.contiguous()
    w = _device.to_dev(vis["weight"].data, torch.float64, dev).contiguous()
    fl = None
    if use_flags:
        fl = _device.to_dev(vis["flags"].data, None, dev)
        if fl.dtype not in kernels._FLAG_DT:
            fl = fl.to(torch.int64)
        fl = fl.contiguous()
    bl = np.asarray(vis.baselines.data)
    a1 = torch.as_tensor(bl[:, 0].astype(np.int32), device=dev)
    a2 = torch.as_tensor(bl[:, 1].astype(np.int32), device=dev)
    gain = _device.to_dev(gt["gain"].data, torch.complex128, dev).contiguous()
    for rs in passes:
        tr = np.full(nvt, -1, dtype=np.int32)
        for r in rs:
            tr[rows[r]] = r
        if not np.any(tr >= 0):
            continue
        kernels.apply_gains(v, w, fl, use_flags, a1, a2, torch.as_tensor(tr, device=dev), gain,
                            inverse)
    _store(vis, "vis", v)
    _store(vis, "weight", w)
    return vis
