"""solve_gaintable on MI355X.

Mirrors reference ``src/ska_sdp_func_python/calibration/solvers.py``:

* ``solve_gaintable`` (:21-145): ValueError for an all-zero model (:56-59),
  ``divide_visibility`` (:61-63), a new gain table if none is given (:70-76),
  per gain row the weighted sums over the row's time window (and over
  frequency when the table has one channel, :82, :99-107), rows without
  weight get gain 1 / weight 0 / residual 0 (:130-133), and finally the
  mean/median gain-amplitude normalisation when not ``phase_only``
  (:135-143).
* the inner solvers (:148-539) run batched over all rows in one call of
  ``sdp_hip_solve_gains``: scalar (npol 1), matrix (npol 4 with crosspol)
  and "nocrossdata" (npol 2, or 4 without crosspol), with the reference's
  channel-coupled convergence, damping 0.5 and refant 0.

The point-source sums (:99-107) are formed on the device; the reference's
dense [nants, nants] matrix (:108-114) is replaced by a canonical packed
baseline order (kernels.canonical_baselines).

Multi-GPU, opt-in with ``shard=True`` (a keyword beyond
the reference's) or SDP_HIP_SHARD=1: with torch.distributed initialised
(more than one rank, every rank calling with the same inputs, which is
checked first) each rank forms the sums and solves a contiguous block of the
gain rows, with no collective in the solve; one all-gather assembles the
table on every rank, and the mean/median normalisation (:135-143) then runs
over the whole table as in the reference.  With ``shard="local"`` every rank
passes its own visibilities (its times) and gets its own rows of the table;
the normalisation is taken over all the ranks' rows (one all-reduce for the
mean, an all-gather of |g| for the median).  By default every rank solves
its own call.
"""

import logging

import numpy as np
import torch

from .. import _device, kernels, parallel
from ..datamodels import create_gaintable_from_visibility

log = logging.getLogger("func-python-logger")


def _windows(vis_time, gain_table):
    """CSR of each gain row's vis times (inclusive xarray slice, solvers.py:84-91)."""
    gtimes = np.asarray(gain_table.time.data, dtype=float)
    interval = np.asarray(gain_table.interval.data, dtype=float)
    idx, ptr = [], [0]
    for row in range(len(gtimes)):
        sel = np.nonzero((vis_time >= gtimes[row] - interval[row] / 2)
                         & (vis_time <= gtimes[row] + interval[row] / 2))[0]
        idx.extend(sel.tolist())
        ptr.append(len(idx))
    ptr = np.asarray(ptr, dtype=np.int32)
    return ptr, np.asarray(idx, dtype=np.int32), np.diff(ptr) > 0


def solve_gaintable(vis, modelvis=None, gain_table=None, phase_only=True, niter=200, tol=1e-6,
                    crosspol=False, normalise_gains="mean", jones_type="T", timeslice=None,
                    shard=None):
    if modelvis is not None:
        mv = modelvis.vis.data
        mx = float(mv.abs().max()) if isinstance(mv, torch.Tensor) else float(np.max(np.abs(mv)))
        if not mx > 0.0:
            raise ValueError("solve_gaintable: Model visibility is zero")
    if phase_only:
        log.debug("solve_gaintable: Solving for phase only")
    else:
        log.debug("solve_gaintable: Solving for complex gain")
    if gain_table is None:
        log.debug("solve_gaintable: creating new gaintable")
        gain_table = create_gaintable_from_visibility(vis, jones_type=jones_type, timeslice=timeslice)
    else:
        log.debug("solve_gaintable: starting from existing gaintable")

    dev = _device.device()
    nants = gain_table.gaintable_acc.nants
    nchan = gain_table.gaintable_acc.nchan
    npol = vis.visibility_acc.npol
    # divide_visibility (solvers.py:61-63) and the per-row sums (:82-107) in
    # one HIP pass, written in StefCal's canonical baseline order
    v = _device.to_dev(vis["vis"].data, None, dev)
    if v.dtype not in (torch.complex64, torch.complex128):
        v = v.to(torch.complex128)
    v = v.contiguous()
    m = None
    if modelvis is not None:
        m = _device.to_dev(modelvis["vis"].data, v.dtype, dev).contiguous()
    w = _device.to_dev(vis["weight"].data, torch.float64, dev).contiguous()
    fl = _device.to_dev(vis["flags"].data, None, dev)
    if fl.dtype not in kernels._FLAG_DT:
        fl = fl.to(torch.int64)
    ptr, tidx, present = _windows(np.asarray(vis.time.data, dtype=float), gain_table)
    for row in np.nonzero(~present)[0]:
        log.warning("Gaintable %s, vis time mismatch %s", gain_table.time.data, vis.time.data)
    # this rank's gain rows [r0, r1) (all of them unsharded)
    nrow_g = len(present)
    sh = parallel.shard_info({"shard": shard})
    parallel.check_replicated(sh, [v, m, w, np.asarray(vis.time.data, dtype=float),
                                  tuple(gain_table["gain"].data.shape)],
                              "solve_gaintable")
    # shard="local": each rank solves the gain table of its OWN visibilities
    # (its time rows); only the mean / median normalisation spans the ranks
    loc = parallel.local_info({"shard": shard})
    parallel.check_replicated(loc, [(nants, nchan, npol)], "solve_gaintable(shard='local')")
    rblocks = [(0, nrow_g)]
    r0, r1 = 0, nrow_g
    if sh:
        rblocks = [parallel.shard_range(nrow_g, r, sh[1]) for r in range(sh[1])]
        r0, r1 = rblocks[sh[0]]
    tidx = tidx[ptr[r0]:ptr[r1]]
    ptr = (ptr[r0:r1 + 1] - ptr[r0]).astype(np.int32)
    present = present[r0:r1]
    bl = np.asarray(vis.baselines.data)
    perm, conj, row_start, ant2 = kernels.canonical_baselines(bl[:, 0], bl[:, 1], nants)
    # autocorrelations go after the canonical baselines: the solver never
    # sees them, but they count in the reference's "any weight" test (:116)
    autos = np.nonzero(bl[:, 0] == bl[:, 1])[0]
    nc = len(perm)
    full_perm = np.concatenate([np.asarray(perm, dtype=np.int64), autos]).astype(np.int32)
    full_conj = np.concatenate([np.asarray(conj, dtype=bool), np.zeros(len(autos), bool)])
    mfl = None
    if modelvis is not None and modelvis["flags"].data is not vis["flags"].data:
        mfl = _device.to_dev(modelvis["flags"].data, None, dev)
    if r1 > r0:
        xb_all, xwt = kernels.point_sums(
            v, m, w, fl.contiguous(), torch.as_tensor(ptr, device=dev),
            torch.as_tensor(tidx if len(tidx) else np.zeros(1, np.int32), device=dev), nchan,
            perm=torch.as_tensor(full_perm, device=dev),
            conj=torch.as_tensor(full_conj.astype(np.uint8), device=dev), model_flags=mfl)
    else:  # more ranks than gain rows: this rank has none
        xb_all = torch.zeros((0, len(full_perm), nchan, npol), dtype=torch.complex128, device=dev)
        xwt = torch.zeros((0, len(full_perm), nchan, npol), dtype=torch.float64, device=dev)
    if len(autos):
        xb_c, xwt_c = xb_all[:, :nc].contiguous(), xwt[:, :nc].contiguous()
    else:
        xb_c, xwt_c = xb_all, xwt

    if npol == 2 or (npol == 4 and not crosspol):
        mode = 2
    elif npol == 4 and crosspol:
        mode = 1
    else:
        mode = 0

    gain_h = gain_table["gain"].data[r0:r1]
    wt_h = gain_table["weight"].data[r0:r1]
    res_h = gain_table["residual"].data[r0:r1]
    gain = _device.to_dev(gain_h, torch.complex128, dev).contiguous().clone()
    gwt = _device.to_dev(wt_h, torch.float64, dev).contiguous().clone()
    if r1 > r0:
        residual, used = kernels.solve_gains(xb_c, xwt_c, gain, gwt, row_start, ant2, mode,
                                             niter=niter, tol=tol, phase_only=phase_only)
    else:
        residual = torch.zeros(res_h.shape, dtype=torch.float64, device=dev)
        used = torch.zeros(0, dtype=torch.int32, device=dev)
    used_h = used.cpu().numpy()
    for row in np.nonzero(used_h > niter)[0]:
        if present[row]:
            log.warning("solve_antenna_gains_itsubs: gain solution failed, retaining gain solutions")

    # rows with no weight at all (solvers.py:116, :130-133) and rows without data
    has_wt = (xwt.reshape(xwt.shape[0], -1).abs() > 0).any(dim=1).cpu().numpy() & present
    empty = torch.as_tensor(~has_wt, device=dev)
    gain = torch.where(empty[:, None, None, None, None], torch.ones_like(gain), gain)
    gwt = torch.where(empty[:, None, None, None, None], torch.zeros_like(gwt), gwt)
    residual = torch.where(empty[:, None, None, None], torch.zeros_like(residual), residual)
    # rows whose times are absent keep their input values (solvers.py:93-97)
    if (~present).any():
        keep = torch.as_tensor(~present, device=dev)
        gain = torch.where(keep[:, None, None, None, None],
                           _device.to_dev(gain_h, torch.complex128, dev), gain)
        gwt = torch.where(keep[:, None, None, None, None],
                          _device.to_dev(wt_h, torch.float64, dev), gwt)
        residual = torch.where(keep[:, None, None, None],
                               _device.to_dev(res_h, torch.float64, dev), residual)
    if sh:
        # the ranks' row blocks assembled on every rank (the solve itself
        # needed no exchange); the normalisation below sees the whole table
        gain = parallel.gather_blocks(gain, rblocks, sh[0], dim=0, group=sh[2])
        gwt = parallel.gather_blocks(gwt, rblocks, sh[0], dim=0, group=sh[2])
        residual = parallel.gather_blocks(residual, rblocks, sh[0], dim=0, group=sh[2])

    if normalise_gains in ["median", "mean"] and not phase_only and loc:
        # the reference normalises over its whole table (solvers.py:135-143):
        # here the table is every rank's rows
        gain = parallel.normalise_gains_global(gain, normalise_gains, loc[2])
    elif normalise_gains in ["median", "mean"] and not phase_only:
        ga = gain.abs().flatten()
        if normalise_gains == "median":
            # numpy median (mean of the two middle values for even counts),
            # not torch.median's lower middle (solvers.py:93-101)
            s = torch.sort(ga).values
            gabs = 0.5 * (s[(ga.numel() - 1) // 2] + s[ga.numel() // 2])
        else:
            gabs = torch.mean(ga)
        gain = gain / gabs

    ref = gain_table["gain"].data
    gain_table["gain"].data = _device.like_input(gain, ref)
    gain_table["weight"].data = _device.like_input(gwt, ref)
    gain_table["residual"].data = _device.like_input(residual, ref)
    return gain_table
