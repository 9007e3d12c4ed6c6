"""predict_ng / invert_ng on MI355X: the reference's ducc0 calls replaced by the
HIP w-stacking NUFFT (libska_sdp_hip: sdp_hip_dirty2ms / sdp_hip_ms2dirty).

Mirrors reference ``src/ska_sdp_func_python/imaging/ng.py``:

* ``predict_ng`` (:38-143): copy with zeroed vis, u and w negated (:80-85),
  MFS when the model has one channel (:95), per (pol, chan) otherwise
  (:113-129), image -> vis polarisation conversion (:131-136), then
  ``shift_vis_to_image(inverse=True)`` (:143); the conversion and the
  phase shift run inside the degridder's write-back (sdp_hip_dirty2ms_vis).
* ``invert_ng`` (:146-294): shift to the image phase centre (:183), flagged
  vis/weights (:191-204), u and w negated (:210-213), MFS when the image has
  one channel and the vis several (:228), PSF puts 1 in pol 0 only
  (:231-233), pols whose vis are all zero are not gridded but their weights
  still enter ``sumwt`` (:238, :258, :267, :289), then ``normalise_sumwt``.
  The phase shift, flag masking, pol conversion, weight conversion and
  weight sums run inside the HIP prologue of sdp_hip_ms2dirty_vis on the
  Visibility's own arrays.  Gridding a pol whose visibilities are all
  zero yields exactly the zero image the reference keeps, so that check
  (ng.py:238) is not a separate pass here.

The image transpose (:102, :257) is folded into the C ABI's output strides.

Multi-GPU, opt-in with ``shard=True`` (a keyword beyond
the reference's) or SDP_HIP_SHARD=1: when torch.distributed is initialised
with more than one rank and every rank calls with the same Visibility and
model (checked first: parallel.check_replicated raises ValueError on every
rank otherwise), the visibility channels are split into contiguous blocks
balanced by the measured cost model (parallel.balanced_channel_blocks).
Without it every rank computes its own call, as the reference does.  invert_ng grids only its block
and combines the partial images and weight sums with one all-reduce each
(the reference's only exchange point, before normalise_sumwt); an MFS invert
with w-stacking instead splits the ROWS into contiguous intervals of w
(parallel.wrow_partition: a rank of small-|w| rows holds few w planes, where
a channel block at the top of a wide band holds them all; SDP_HIP_SHARD=chan
keeps channel blocks); predict_ng predicts its block and all-gathers the
channel blocks.  Every rank returns
the reference's full result.

Pre-sharded mode, ``shard="local"`` (or SDP_HIP_SHARD=local): every rank
passes its OWN block of one observation -- its channels, or its rows (e.g.
an interval of w from parallel.wrow_partition) -- and only the image
geometry is checked to agree.  invert_ng grids the rank's block and
all-reduces the partial image and weight sums before normalise_sumwt
(ng.py:288-292), so every rank returns the whole observation's image;
predict_ng predicts the rank's block with no exchange.  A block larger than
one NUFFT call holds (SDP_HIP_MAX_CALL_GVIS, default 1.8 Gvis) is gridded in
channel batches through one set of resident w planes
(sdp_hip_ms2dirty_vis_batch).
Kwargs ``epsilon`` (default 1e-12), ``do_wstacking`` (True), ``threads``
and ``verbosity`` are accepted as in the reference; ``threads`` is ignored
(one GPU per process).  epsilon < 1e-7 runs the fp64 NUFFT (as ducc0 with
double_precision_accumulation); ``precision="fp32"`` (beyond the reference)
serves such requests with the fp32 NUFFT at its floor (W = 8, ~1e-6).
"""

import contextlib
import logging
import os
import threading

import numpy as np
import torch

from .. import _device, kernels, parallel
from ..datamodels import Image, pol_conversion_matrix
from .base import normalise_sumwt, shift_lmn

log = logging.getLogger("func-python-logger")


def _vis_to_im(model, freq):
    return np.round(model.image_acc.wcs.sub([4]).wcs_world2pix(np.asarray(freq), 0)[0]).astype(int)


def _channel_runs(vis_to_im, lo, hi):
    """(image channel, first, end) of each run of consecutive visibility
    channels in [lo, hi) that map to the same image channel."""
    runs = []
    for v in range(lo, hi):
        ichan = int(vis_to_im[v])
        if runs and runs[-1][0] == ichan:
            runs[-1][2] = v + 1
        else:
            runs.append([ichan, v, v + 1])
    return [tuple(r) for r in runs]


def _image_geometry(model, **scalars):
    """What every rank of a shard="local" call must agree on: the image shape,
    its WCS (reference pixels, increments, values) and polarisation frame,
    and the call's scalar options (epsilon, do_wstacking, dopsf, ...): ranks
    that pass different ones would all-reduce images that do not match."""
    w = model.image_acc.wcs.wcs
    frame = model.image_acc.polarisation_frame
    text = repr((str(getattr(frame, "type", frame)), sorted(scalars.items()))).encode()
    return [tuple(model["pixels"].data.shape), np.asarray(w.crpix, dtype=float),
            np.asarray(w.cdelt, dtype=float), np.asarray(w.crval, dtype=float),
            np.frombuffer(text, dtype=np.uint8)]


def _pixsize(model):
    return float(np.abs(np.radians(model.image_acc.wcs.wcs.cdelt[0])))


_SIDE = {}


def _side_stream(dev):
    """The second stream of a pipelined invert (one per device)."""
    s = _SIDE.get(dev.index)
    if s is None:
        s = _SIDE[dev.index] = torch.cuda.Stream(dev)
    return s


_COPY = {}
_HOST_LOOKAHEAD = 2  # time blocks a streamed host invert copies ahead of its gridding


def _copy_stream(dev):
    """The host-to-device copy stream of a streamed host-resident invert."""
    s = _COPY.get(dev.index)
    if s is None:
        s = _COPY[dev.index] = torch.cuda.Stream(dev)
    return s


def _host_row_blocks(sbvis, dev, single_call, dopsf, lo, hi, vnchan, nvis, max_call):
    """Time blocks for streaming a host-resident Visibility through one NUFFT
    call, or None.  A host Visibility's vis / weight / flag arrays cross PCIe
    before any compute (~4 GB for C2); cut by time (contiguous slices), block
    k + 1 is copied on a copy stream while block k grids, as one batch
    sequence through one set of w planes.  SDP_HIP_HOST_BLOCKS (default 4;
    0 or 1 = copy everything first)."""
    nb = int(os.environ.get("SDP_HIP_HOST_BLOCKS", "4"))
    ntimes = sbvis.vis.shape[0]
    arrs = (sbvis.vis.data, sbvis.imaging_weight.data, sbvis.flags.data)
    if (dev.type != "cuda" or not single_call or dopsf or nb <= 1 or (lo, hi) != (0, vnchan)
            or not all(isinstance(a, np.ndarray) for a in arrs)):
        return None
    nb = min(ntimes, max(nb, -(-nvis // max_call)))
    if nb <= 1:
        return None
    return [ntimes * i // nb for i in range(nb + 1)]


def _rank_rows(uvw, freq, npix, pixsize, epsilon, precision, shard):
    """This rank's rows of an MFS w-stacked invert: an interval of the rows'
    w (RASCIL's sign, u and w negated) cut by parallel.wrow_partition over
    the band's plane spacing (kernels.wstack_layout)."""
    b = [float(uvw[:, 2].min()), float(uvw[:, 2].max()), float(uvw[:, 0].abs().max()),
         float(uvw[:, 1].abs().max()), float(np.min(freq)), float(np.max(freq))]
    lay = kernels.wstack_layout(b, npix, npix, pixsize, pixsize, epsilon, True, flip_uw=True,
                                precision=precision)
    order, cuts, _ = parallel.wrow_partition(-uvw[:, 2].cpu().numpy(), freq, shard[1], lay["dw"],
                                             lay["support"])
    return torch.as_tensor(order[cuts[shard[0]]:cuts[shard[0] + 1]], device=uvw.device)


def predict_ng(bvis, model, **kwargs):
    """Predict visibilities from a model Image (reference ng.py:38)."""
    if model is None:
        return bvis
    assert isinstance(model, Image) or hasattr(model, "image_acc"), model
    assert model.image_acc.is_canonical()

    epsilon = kwargs.get("epsilon", 1e-12)
    do_wstacking = kwargs.get("do_wstacking", True)
    verbosity = kwargs.get("verbosity", 0)
    precision = kwargs.get("precision")

    dev = _device.device()
    freq = np.asarray(bvis.frequency.data, dtype=float)
    nrows, nbaselines, vnchan, vnpol = bvis.vis.shape
    uvw = _device.to_dev(bvis.uvw.data, torch.float64, dev).reshape(nrows * nbaselines, 3)
    uvw = torch.nan_to_num(uvw).contiguous()
    shard = parallel.shard_info(kwargs)
    parallel.check_replicated(shard, [uvw, freq, model["pixels"].data], "predict_ng")
    # shard="local": each rank predicts its own block, no exchange; the model
    # must be the same on every rank
    loc = parallel.local_info(kwargs)
    parallel.check_replicated(
        loc, _image_geometry(model, epsilon=float(epsilon), do_wstacking=bool(do_wstacking),
                             precision=precision) + [model["pixels"].data],
        "predict_ng(shard='local')")
    blocks = [(0, vnchan)]
    lo, hi = 0, vnchan
    if shard:
        blocks = parallel.balanced_channel_blocks(freq, shard[1])
        lo, hi = blocks[shard[0]]
    freq_t = _device.to_dev(freq[lo:hi], torch.float64, dev)

    pixels = _device.to_dev(model["pixels"].data, torch.float64, dev)
    m_nchan, m_npol, ny, nx = pixels.shape
    assert m_npol == vnpol
    pixsize = _pixsize(model)
    vis_to_im = _vis_to_im(model, freq)
    # image -> vis pol frame (ng.py:131-136) fused into the write-back: image
    # pol p adds column p of the conversion matrix times its prediction to
    # every vis pol; the result lands in the output's own dtype and layout
    conv = pol_conversion_matrix(model.image_acc.polarisation_frame,
                                 bvis.visibility_acc.polarisation_frame)
    src = bvis["vis"].data
    lmn = shift_lmn(bvis, model)  # shift_vis_to_image(inverse=True) (ng.py:143), in-kernel
    vdt = src.dtype if _device.is_device(src) and src.is_complex() else torch.complex128
    vist = torch.empty((nrows * nbaselines, hi - lo, vnpol), dtype=vdt, device=dev)

    def coef(p):
        if conv is None:
            c = np.zeros(vnpol, complex)
            c[p] = 1.0
            return c
        return conv[:, p]

    info = None
    if m_nchan == 1 and vnpol > 1 and hi > lo:
        # every image pol in one call: one bucketing, one write-back
        _, info = kernels.dirty2ms_vis_pols(uvw, freq_t, pixels[0], vist,
                                            [coef(p) for p in range(vnpol)], pixsize, pixsize,
                                            epsilon, do_wstacking, flip_uw=True,
                                            dirty_strides=(pixels.stride(1), 1, nx),
                                            npix=(nx, ny), shift_lmn=lmn, precision=precision)
    for vpol in range(vnpol if hi > lo and not (m_nchan == 1 and vnpol > 1) else 0):
        if m_nchan == 1:
            _, info = kernels.dirty2ms_vis(uvw, freq_t, pixels[0, vpol], vist, coef(vpol), pixsize,
                                           pixsize, epsilon, do_wstacking, flip_uw=True,
                                           dirty_strides=(1, nx), npix=(nx, ny),
                                           accumulate=vpol > 0, shift_lmn=lmn,
                                           precision=precision)
        else:
            for vchan in range(lo, hi):
                img = pixels[int(vis_to_im[vchan]), vpol]
                c = vchan - lo
                _, info = kernels.dirty2ms_vis(uvw, freq_t[c:c + 1], img,
                                               vist[:, c:c + 1, :], coef(vpol), pixsize,
                                               pixsize, epsilon, do_wstacking, flip_uw=True,
                                               dirty_strides=(1, nx), npix=(nx, ny),
                                               accumulate=vpol > 0, shift_lmn=lmn,
                                           precision=precision)
    if verbosity and info is not None:
        log.info("predict_ng: %s", info)
    if shard:
        # every rank's channel block, assembled on every rank
        vist = parallel.gather_blocks(vist, blocks, shard[0], dim=1, group=shard[2])

    vis = vist.reshape(nrows, nbaselines, vnchan, vnpol)
    # the reference's bvis.copy(deep=True, zero=True) (ng.py:77), with the
    # predicted visibilities in place of the zeroed copy
    out = _device.like_input(vis, src)
    if isinstance(out, np.ndarray) and out.dtype != np.asarray(src).dtype:
        out = out.astype(np.asarray(src).dtype)
    newbvis = bvis._copy_with(deep=True, replace={"vis": out})
    if lmn is not None:
        # the reference's shift_vis_to_image relabels the phase centre
        # (imaging/base.py:90)
        newbvis.attrs["phasecentre"] = model.image_acc.phasecentre
    return newbvis


def invert_ng(bvis, model, dopsf=False, normalise=True, **kwargs):
    """Invert visibilities to an (Image, sumwt) pair (reference ng.py:146)."""
    assert isinstance(model, Image) or hasattr(model, "image_acc"), model
    assert model.image_acc.is_canonical()

    epsilon = kwargs.get("epsilon", 1e-12)
    do_wstacking = kwargs.get("do_wstacking", True)
    verbosity = kwargs.get("verbosity", 0)
    precision = kwargs.get("precision")

    dev = _device.device()
    nchan, npol, ny, nx = model["pixels"].data.shape
    image = torch.zeros((nchan, npol, ny, nx), dtype=torch.float64, device=dev)
    shard = parallel.shard_info(kwargs)
    loc = parallel.local_info(kwargs)
    # the reference's deep copy + zero fill (ng.py:173, :218) without
    # copying the model's pixels
    im = model.copy(deep=True, data=image)
    # shift_vis_to_image (ng.py:183) is applied inside the kernel's prologue
    lmn = None if dopsf else shift_lmn(bvis, im)
    sbvis = bvis
    freq = np.asarray(sbvis.frequency.data, dtype=float)
    nrows, nbaselines, vnchan, vnpol = sbvis.vis.shape
    nrow = nrows * nbaselines
    # this rank's visibility channels [lo, hi) (all of them unsharded), or
    # for an MFS w-stacked invert its rows (an interval of w, all channels)
    lo, hi = 0, vnchan
    # MFS: one image channel collecting several visibility channels.  In the
    # pre-sharded mode a rank's block may hold a single channel of a
    # many-channel observation, so there an MFS image alone decides it
    mfs = nchan == 1 and (vnchan > 1 or loc is not None)
    uvw = _device.to_dev(sbvis.uvw.data, torch.float64, dev).reshape(nrow, 3).contiguous()
    parallel.check_replicated(
        shard, [uvw, freq, sbvis.imaging_weight.data, None if dopsf else sbvis.vis.data,
                model["pixels"].data.shape], "invert_ng")
    # shard="local": each rank passes its own block; the image geometry and
    # the call's options must agree across the ranks
    parallel.check_replicated(
        loc, _image_geometry(model, epsilon=float(epsilon), do_wstacking=bool(do_wstacking),
                             dopsf=bool(dopsf), normalise=bool(normalise), precision=precision),
        "invert_ng(shard='local')")
    rows = None
    if shard and mfs and do_wstacking and parallel.shard_mode() != "chan":
        rows = _rank_rows(uvw, freq, nx, _pixsize(im), epsilon, precision, shard)
    elif shard:
        lo, hi = parallel.balanced_channel_blocks(freq, shard[1])[shard[0]]
    nloc = hi - lo

    def local(arr, dtype=None):
        # the rank's slice: rows gathered on the host before the copy when
        # the Visibility is host-resident (only 1/N of it crosses PCIe)
        a = arr[:, :, lo:hi]
        if rows is None:
            return _device.to_dev(a, dtype, dev).reshape(nrow, nloc, vnpol)
        a = a.reshape((nrow,) + tuple(a.shape[2:]))
        if isinstance(a, np.ndarray):
            return _device.to_dev(a[rows.cpu().numpy()], dtype, dev)
        return _device.to_dev(a, dtype, dev)[rows]

    max_call = max(1, int(float(os.environ.get("SDP_HIP_MAX_CALL_GVIS", "1.8")) * 1e9))
    tcuts = None
    if rows is None and uvw.shape[0] > 0:
        tcuts = _host_row_blocks(sbvis, dev, mfs and npol == 1, dopsf, lo, hi, vnchan,
                                 nrow * vnchan, max_call)

    def typed(flags, wgt, ms):
        if flags.dtype not in kernels._FLAG_DT:
            flags = flags.to(torch.int64)
        if wgt.dtype not in (torch.float32, torch.float64):
            wgt = wgt.to(torch.float64)
        if ms is not None and ms.dtype not in (torch.complex64, torch.complex128):
            ms = ms.to(torch.complex128)
        return flags, wgt, ms

    # The Visibility's own arrays, read in place by the fused prologue of
    # sdp_hip_ms2dirty_vis: flag masking (ng.py:191, :202), the pol-frame
    # conversion (ng.py:193-198) as one matrix row per image pol, f64 weights
    # and the weight sums (ng.py:258, :289) -- no O(Nvis) passes here.
    # (A streamed host Visibility copies them block by block below.)
    flags = wgt = ms = None

    def whole_arrays():
        nonlocal flags, wgt, ms
        flags, wgt, ms = typed(local(sbvis.flags.data), local(sbvis.imaging_weight.data),
                               None if dopsf else local(sbvis.vis.data))

    if tcuts is None:
        whole_arrays()
    conv = pol_conversion_matrix(bvis.visibility_acc.polarisation_frame,
                                 im.image_acc.polarisation_frame)
    if rows is not None:
        uvw = uvw[rows].contiguous()
    freq_t = _device.to_dev(freq[lo:hi], torch.float64, dev)

    npixdirty = nx
    pixsize = _pixsize(im)
    sumwt_d = torch.zeros((nchan, npol), dtype=torch.float64, device=dev)
    vis_to_im = _vis_to_im(model, freq)

    # the (pol, channel) images the reference loops over (ng.py:236-289): all
    # pols of the band for MFS; for a cube, one call per image pol and run of
    # consecutive visibility channels that map to one image channel.  The
    # reference adds one ducc0 call per visibility channel into im[ichan]
    # (ng.py:259-289); the sum is linear in the visibilities, so a run's
    # channels grid as one call into the same image and weight sum (C2 as a
    # 16-channel cube: 16 calls of 4 channels instead of 64 of one).
    nrow_loc = uvw.shape[0]
    if mfs:
        calls = [(pol, slice(0, nloc), 0) for pol in range(npol if nloc > 0 else 0)]
    else:
        calls = [(pol, slice(a - lo, b - lo), ichan)
                 for ichan, a, b in _channel_runs(vis_to_im, lo, hi) for pol in range(npol)]
    if nrow_loc == 0:
        calls = []  # (a rank with no rows: its share of the exchange is zeros)
    grid_calls = [c for c in calls if not (dopsf and c[0] != 0)]
    # A call over more visibilities than one NUFFT call holds (records,
    # 2^32 limit: SDP_HIP_MAX_CALL_GVIS, default 1.8 Gvis -- a C4 rank's
    # block) grids its channels in batches through one set of resident w
    # planes (sdp_hip_ms2dirty_vis_batch); the reference makes one ducc0 call
    # over all channels (ng.py:240-256).
    def batches(chans):
        n = chans.stop - chans.start
        nb = min(n, max(1, -(-nrow_loc * n // max_call)))
        cuts = [chans.start + n * i // nb for i in range(nb + 1)]
        return [slice(a, e) for a, e in zip(cuts[:-1], cuts[1:])]

    batched = tcuts is not None or any(len(batches(c[1])) > 1 for c in grid_calls)
    # The pols of one image channel share one bucketing: the first pol keeps
    # it, the others re-run only the value pass (SDP_HIP_KEEP_BUCKETS /
    # SDP_HIP_REUSE_BUCKETS; C2 4 pols 54.0 ms against 59.7 pipelined, bench
    # api object).  Otherwise two or more NUFFT calls -- a single-pol cube's
    # channel runs -- are pipelined over two streams and the library's two
    # scratch slots, so one call's bucketing runs under the other's gridding
    # and FFT.  The stream is picked by the OUTPUT (image channel, pol), not
    # by the call's position: the image and weight-sum accumulation is a
    # plain read-modify-write, so every call into one target stays on one
    # stream.  SDP_HIP_OVERLAP=0 keeps every call on one stream.
    # (not at fp64: a kept bucketing is single-level, whose unpadded
    # records only the VALU fp64 gridder reads -- the pols then run the
    # two-level sort and the MFMA gridder each, pipelined over two streams)
    share = npol > 1 and not dopsf and not batched and not kernels.is_fp64(epsilon, precision)
    overlap = len(grid_calls) > 1 and not share and not batched and dev.type == "cuda" and \
        os.environ.get("SDP_HIP_OVERLAP", "1") != "0"
    main = torch.cuda.current_stream(dev) if overlap else None
    side = _side_stream(dev) if overlap else None
    if overlap:
        side.wait_stream(main)
    lane_of = {}
    for pol, _, ichan in grid_calls:
        lane_of.setdefault((ichan, pol), len(lane_of) % 2)

    def grid_streamed(pol, chans, ichan):
        """One call over time blocks of a host Visibility: a copy thread moves
        the blocks to the device on the copy stream (a pageable copy blocks
        its host thread, not the GPU) while this thread grids the blocks
        already there, one batch sequence through one set of resident w
        planes (sdp_hip_ms2dirty_vis_batch).  The copier runs at most
        _HOST_LOOKAHEAD blocks ahead of the gridding (so the device holds at
        most that many blocks beyond the one gridding) and stops when the
        gridding ends or fails.  Returns False, with nothing gridded, when the
        w planes do not all fit in device memory at once (a batch sequence
        needs them resident): the caller then copies everything first and
        grids in one call, whose planes are chunked."""
        sw = sumwt_d[ichan, pol:pol + 1]
        coef = None if conv is None else conv[pol]
        main_s, cs = torch.cuda.current_stream(dev), _copy_stream(dev)
        nbl = sbvis.vis.shape[1]
        bounds = kernels.uvw_bounds(uvw, freq_t)
        cs.wait_stream(main_s)
        nblk = len(tcuts) - 1
        got = [None] * nblk
        ready = [threading.Event() for _ in range(nblk)]
        slots = threading.Semaphore(_HOST_LOOKAHEAD)
        stop = threading.Event()

        def copier():
            try:
                with torch.cuda.device(dev), torch.cuda.stream(cs):
                    for i in range(nblk):
                        slots.acquire()
                        if stop.is_set():
                            return
                        t0, t1 = tcuts[i], tcuts[i + 1]
                        n = (t1 - t0) * nbl
                        ts = typed(*(_device.to_dev(a[t0:t1], None, dev).reshape(n, vnchan, vnpol)
                                     for a in (sbvis.flags.data, sbvis.imaging_weight.data,
                                               sbvis.vis.data)))
                        ev = torch.cuda.Event()
                        ev.record(cs)
                        got[i] = (ts, ev)
                        ready[i].set()
            except BaseException as e:  # noqa: BLE001 -- re-raised by the gridding thread
                for i in range(nblk):
                    if got[i] is None:
                        got[i] = e
                    ready[i].set()

        th = threading.Thread(target=copier, daemon=True)
        th.start()
        try:
            for i in range(nblk):
                ready[i].wait()
                if isinstance(got[i], BaseException):
                    raise got[i]
                (fl, wg, vs), ev = got[i]
                got[i] = None
                main_s.wait_event(ev)
                for t in (fl, wg, vs):
                    t.record_stream(main_s)
                r0, r1 = tcuts[i] * nbl, tcuts[i + 1] * nbl
                try:
                    _, info = kernels.ms2dirty_vis(
                        uvw[r0:r1], freq_t, vs, pol, wg[:, :, pol], fl, coef, npixdirty,
                        npixdirty, pixsize, pixsize, epsilon, do_wstacking, flip_uw=True,
                        out=image[ichan, pol], out_strides=(1, nx), accumulate=True, sumwt=sw,
                        shift_lmn=lmn, precision=precision, bounds=bounds, first=i == 0,
                        last=i == nblk - 1)
                except ValueError as e:
                    # (raised by the first batch's plan, before any gridding
                    # or weight sum)
                    if i == 0 and "do not all fit" in str(e):
                        log.info("invert_ng: w planes exceed device memory, host Visibility "
                                 "copied whole instead of streamed")
                        return False
                    raise
                if verbosity:
                    log.info("invert_ng: %s", info)
                del fl, wg, vs
                slots.release()
        finally:
            stop.set()
            slots.release()  # (wakes a copier waiting for a slot)
            th.join()
            got.clear()
        return True

    def grid_pol(pol, chans, ichan, first_pol):
        nonlocal tcuts
        if tcuts is not None:
            if grid_streamed(pol, chans, ichan):
                return
            tcuts = None
            whole_arrays()
        sw = sumwt_d[ichan, pol:pol + 1]
        if dopsf and pol != 0:
            # PSF: pol 0 holds unit visibilities, the others are zero and are
            # not gridded (ng.py:231-233, :238); their weights still count
            m = 1 - flags[:, chans, pol].to(torch.float64)
            sw += (wgt[:, chans, pol].to(torch.float64) * m).sum()
            return
        coef = None if (dopsf or conv is None) else conv[pol]
        lane = lane_of[(ichan, pol)] if overlap else 0
        ctx = torch.cuda.stream(side if lane else main) if overlap else contextlib.nullcontext()
        parts = batches(chans)
        seq = {}
        if len(parts) > 1:
            seq = {"bounds": kernels.uvw_bounds(uvw, freq_t[chans])}
        with ctx:
            for i, part in enumerate(parts):
                if seq:
                    seq.update(first=i == 0, last=i == len(parts) - 1)
                _, info = kernels.ms2dirty_vis(
                    uvw, freq_t[part], None if dopsf else ms[:, part, :], pol, wgt[:, part, pol],
                    flags[:, part, :], coef, npixdirty, npixdirty, pixsize, pixsize, epsilon,
                    do_wstacking, flip_uw=True, out=image[ichan, pol], out_strides=(1, nx),
                    accumulate=True, sumwt=sw, shift_lmn=lmn, keep_buckets=share and first_pol,
                    reuse_buckets=share and not first_pol, precision=precision, slot=lane, **seq)
                if verbosity:
                    log.info("invert_ng: %s", info)

    def grid_pols(chans, ichan):
        """Every image pol of one image channel in one library call
        (sdp_hip_ms2dirty_vis_pols): one bucketing and one value pass that
        reads each visibility's pols, flags and weights once, then each
        pol's gridding and FFT -- the results of one ms2dirty_vis call per
        pol sharing a kept bucketing (C2 4 pols: 5.7 ms value pass per pol)."""
        (part,) = batches(chans)
        _, info = kernels.ms2dirty_vis_pols(
            uvw, freq_t[part], ms[:, part, :], wgt[:, part, :npol], flags[:, part, :],
            None if conv is None else [conv[p] for p in range(npol)], npixdirty, npixdirty,
            pixsize, pixsize, epsilon, do_wstacking, flip_uw=True, out=image[ichan],
            out_strides=(image.stride(1), 1, nx), accumulate=True, sumwt=sumwt_d[ichan, :npol],
            shift_lmn=lmn, precision=precision)
        if verbosity:
            log.info("invert_ng: %s", info)

    if share and tcuts is None and ms.shape[2] >= npol and wgt.shape[2] >= npol:
        done = set()
        for _, chans, ichan in calls:
            key = (chans.start, chans.stop, ichan)
            if key not in done:
                done.add(key)
                grid_pols(chans, ichan)
    else:
        for pol, chans, ichan in calls:
            grid_pol(pol, chans, ichan, pol == 0)
    if overlap:
        main.wait_stream(side)
    if shard or loc:
        # the one exchange: partial images and weight sums of the ranks'
        # blocks (before normalise_sumwt, ng.py:292)
        grp = (shard or loc)[2]
        parallel.all_reduce_sum(image, grp)
        parallel.all_reduce_sum(sumwt_d, grp)
    sumwt = sumwt_d.cpu().numpy()

    im["pixels"].data = image
    if normalise:
        im = normalise_sumwt(im, sumwt)
    im["pixels"].data = _device.like_input(im["pixels"].data, bvis["vis"].data)
    return im, sumwt
