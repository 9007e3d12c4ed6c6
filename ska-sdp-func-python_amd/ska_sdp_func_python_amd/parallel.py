"""Multi-GPU invert: visibilities sharded by channel, one all-reduce.

One process per GPU (torchrun); the process group is RCCL ("nccl") on
MI355X, gloo in the CPU tests.  Each rank grids its channel shard with the
HIP w-stacking NUFFT into a partial fp64 dirty image and a partial sum of
weights, then a single ``all_reduce(SUM)`` of the image (npix^2 x 8 B) and
of sumwt over xGMI combines them before the normalisation -- the reference's
invert_ng/normalise_sumwt (imaging/ng.py:235-292, imaging/base.py:95-128)
split at its only exchange point.  Each rank chooses its
own w planes, so no uv-grid exchange is needed.
"""

import numpy as np
import torch
import torch.distributed as dist


def shard_range(n, rank, world):
    """Contiguous [lo, hi) block of n items for ``rank`` of ``world``."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def interleaved_channels(nchan_total, rank, world):
    """Channel indices rank, rank+world, ... (every shard spans the band)."""
    return np.arange(rank, nchan_total, world)


def _gridder():
    from . import kernels
    return kernels.ms2dirty


def invert_sharded(uvw, freq, vis, wgt, npix, cell, epsilon=1e-7, do_wstacking=True,
                   flip_uw=True, normalise=True, group=None, grid_fn=None, out=None):
    """Invert this rank's shard and all-reduce.

    uvw [nrow,3], freq [nchan_shard], vis/wgt [nrow, nchan_shard] are the
    rank-local arrays.  Returns (dirty [npix, npix] in RASCIL [y, x] order,
    sumwt) identical on every rank.
    """
    grid_fn = grid_fn or _gridder()
    dev = uvw.device
    if out is None:
        out = torch.zeros((npix, npix), dtype=torch.float64, device=dev)
    else:
        out.zero_()
    if freq.numel() > 0 and uvw.shape[0] > 0:
        grid_fn(uvw, freq, vis, wgt, npix, npix, cell, cell, epsilon, do_wstacking,
                flip_uw=flip_uw, out=out, out_strides=(1, npix), accumulate=True)
    sumwt = (wgt.sum() if wgt is not None else torch.tensor(float(vis.numel()), device=dev))
    sumwt = sumwt.to(torch.float64).reshape(1)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(sumwt, op=dist.ReduceOp.SUM, group=group)
    if normalise:
        s = float(sumwt.item())
        if s > 0:
            out /= s
        else:
            out.zero_()
    return out, sumwt
