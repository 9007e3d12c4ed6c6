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


def shard_mode():
    """SDP_HIP_SHARD: unset / "0" off, "chan" channel blocks everywhere, any
    other value rows by w for MFS w-stacked inverts and channel blocks for
    the rest."""
    import os
    return os.environ.get("SDP_HIP_SHARD", "0")


def shard_info(kwargs=None):
    """(rank, world, group) when the reference-shaped API (invert_ng,
    predict_ng, solve_gaintable) should shard its work across the ranks of
    the default process group.

    Sharding is OPT-IN: the kwarg ``shard=True`` (beyond the reference's
    signature) or SDP_HIP_SHARD=1 / chan, with torch.distributed initialised
    over more than one rank and every rank calling with the same (replicated)
    inputs.  Each rank then computes its share and one collective combines
    the shares, so every rank returns the reference's full result.  By
    default each rank computes its own call independently, as the reference
    does: ranks of a data-parallel pipeline pass different data.  The
    entry points check replication with :func:`check_replicated` before they
    split anything."""
    import os
    want = None if kwargs is None else kwargs.get("shard")
    if want is None:
        env = os.environ.get("SDP_HIP_SHARD", "0")
        want = env not in ("", "0", "local")
    if not want or want == "local":
        return None
    return _group_info()


def _group_info():
    if not (dist.is_available() and dist.is_initialized()):
        return None
    world = dist.get_world_size()
    if world <= 1:
        return None
    return dist.get_rank(), world, None


def local_info(kwargs=None):
    """(rank, world, group) for the PRE-SHARDED mode, ``shard="local"`` (or
    SDP_HIP_SHARD=local), with torch.distributed initialised over more than
    one rank: every rank passes its OWN block of one observation (its
    channels, or its rows -- e.g. an interval of w, wrow_partition) and the
    calls combine the blocks at the reference's exchange points: invert_ng
    all-reduces the partial images and weight sums before normalise_sumwt
    (ng.py:288-292); predict_ng predicts each block with no exchange;
    solve_gaintable solves each rank's gain rows and normalises the gains
    over the whole table (solvers.py:135-143).  Nothing is replicated, so the
    visibilities of a band too large for one GPU (C4: 13.4 Gvis) never sit on
    one device.  None otherwise."""
    import os
    want = None if kwargs is None else kwargs.get("shard")
    if want is None:
        want = os.environ.get("SDP_HIP_SHARD", "0")
    if want != "local":
        return None
    return _group_info()


_HASH_CHUNK = 1 << 24  # bytes hashed per step (bounds the temporaries)


def _byte_hash(a):
    """Two int64 sums over the array's bytes taken as 32-bit words: plain and
    position-weighted (weight = word index mod 65521, plus 1), both modulo
    2^64.  Computed in chunks of _HASH_CHUNK bytes on the array's own device,
    so the temporaries stay small whatever the array's size; identical bytes
    (NaNs included) hash identically."""
    if isinstance(a, torch.Tensor):
        flat = a.reshape(-1)
        item = flat.element_size()
        step = max(1, _HASH_CHUNK // item)
        s0 = torch.zeros((), dtype=torch.int64, device=a.device)
        s1 = torch.zeros((), dtype=torch.int64, device=a.device)
        word0 = 0
        for i in range(0, flat.numel(), step):
            b = flat[i:i + step].contiguous().view(torch.uint8)
            pad = (-b.numel()) % 4
            if pad:
                b = torch.cat([b, b.new_zeros(pad)])
            w = b.view(torch.int32).to(torch.int64)
            idx = (torch.arange(word0, word0 + w.numel(), device=a.device) % 65521) + 1
            s0 += w.sum()
            s1 += (w * idx).sum()
            word0 += w.numel()
        return [int(s0), int(s1)]
    flat = np.asarray(a).reshape(-1)
    step = max(1, _HASH_CHUNK // max(flat.itemsize, 1))
    s0 = s1 = 0
    word0 = 0
    for i in range(0, flat.size, step):
        b = np.ascontiguousarray(flat[i:i + step]).view(np.uint8)
        if b.size % 4:
            b = np.concatenate([b, np.zeros((-b.size) % 4, np.uint8)])
        w = b.view(np.int32).astype(np.int64)
        idx = (np.arange(word0, word0 + w.size, dtype=np.int64) % 65521) + 1
        with np.errstate(over="ignore"):
            s0 = (s0 + int(w.sum(dtype=np.int64))) & 0xFFFFFFFFFFFFFFFF
            s1 = (s1 + int((w * idx).sum(dtype=np.int64))) & 0xFFFFFFFFFFFFFFFF
        word0 += w.size
    return [s0 - (1 << 64) if s0 >= 1 << 63 else s0, s1 - (1 << 64) if s1 >= 1 << 63 else s1]


def _fingerprint(arrays):
    """int64 vector: per array its rank, shape and (for arrays) a hash of its
    bytes (_byte_hash), in a fixed order."""
    out = []
    for a in arrays:
        if a is None:
            out += [-1]
            continue
        if isinstance(a, (tuple, list)) and all(isinstance(s, (int, np.integer)) for s in a):
            out += [len(a)] + [int(s) for s in a]  # a shape
            continue
        t = a if isinstance(a, torch.Tensor) else np.asarray(a)
        out += [t.ndim] + [int(s) for s in t.shape]
        if t.size == 0 if isinstance(t, np.ndarray) else t.numel() == 0:
            continue
        out += _byte_hash(t)
    return torch.tensor(out, dtype=torch.int64)


def check_replicated(shard, arrays, what):
    """Raise ValueError on EVERY rank unless every rank of ``shard`` passed
    the same arrays (shapes and byte hashes agree): a sharded call splits
    one replicated problem, and ranks that pass their own data would
    otherwise combine unrelated partial results (or hang in a collective of
    mismatched shapes).  One small all-reduce pair of int64 vectors."""
    if not shard:
        return
    fp = _fingerprint(arrays)
    dev = torch.device("cpu")
    if dist.get_backend(shard[2]) != "gloo":  # RCCL takes device tensors only
        dev = torch.device("cuda", torch.cuda.current_device())
    fp = fp.to(dev)
    # the fingerprints' lengths first: a shape mismatch changes the length
    n = torch.tensor([len(fp), -len(fp)], dtype=torch.int64, device=dev)
    dist.all_reduce(n, op=dist.ReduceOp.MAX, group=shard[2])
    same = int(n[0]) == -int(n[1])
    if same:
        hi = fp.clone()
        lo = -fp
        dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=shard[2])
        dist.all_reduce(lo, op=dist.ReduceOp.MAX, group=shard[2])
        same = bool(torch.equal(hi, -lo))
    if not same:
        raise ValueError(f"{what}: sharding needs the same inputs on every rank (the ranks "
                         "passed different visibilities, models, tables or image geometries); "
                         "call without sharding to process each rank's own data")


def _host_staged(group, t):
    """gloo (the CPU backend) is given host copies of device tensors."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_reduce_sum(t, group=None):
    """In-place SUM all-reduce of a real or complex tensor (complex as its
    real view, which every backend accepts)."""
    x = torch.view_as_real(t) if t.is_complex() else t
    if _host_staged(group, x):
        h = x.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        x.copy_(h)
    else:
        dist.all_reduce(x, op=dist.ReduceOp.SUM, group=group)
    return t


def gather_blocks(local, blocks, rank, dim, group=None):
    """Every rank's contiguous block [lo, hi) of axis ``dim`` (blocks =
    [(lo, hi)] per rank, ``local`` = this rank's block) assembled into the
    full tensor on every rank: one all_gather of the blocks padded to the
    largest (complex tensors as their real view)."""
    width = max(hi - lo for lo, hi in blocks)
    x = local.movedim(dim, 0)
    pad = torch.zeros((width,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[:x.shape[0]] = x
    if pad.is_complex():
        pad = torch.view_as_real(pad)
    dev = pad.device
    if _host_staged(group, pad):
        pad = pad.cpu()
    parts = [torch.empty_like(pad) for _ in blocks]
    dist.all_gather(parts, pad.contiguous(), group=group)
    parts = [q.to(dev) for q in parts]
    if local.is_complex():
        parts = [torch.view_as_complex(q) for q in parts]
    full = torch.cat([q[:hi - lo] for q, (lo, hi) in zip(parts, blocks)], dim=0)
    return full.movedim(0, dim).contiguous()


def shard_range(n, rank, world):
    """Contiguous [lo, hi) block of n items for ``rank`` of ``world``."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def interleaved_channels(nchan_total, rank, world):
    """Channel indices rank, rank+world, ... (every shard spans the band)."""
    return np.arange(rank, nchan_total, world)


# Cost model of one rank's invert of a contiguous channel block of the C4
# band (SKA-LOW 512 stations x 400 times, 8192^2 image, 16384^2 grid): a
# non-negative least-squares fit to the per-rank stage times of the 8-way
# partition measured on one MI355X with the round-3 kernels
# (profiles/r03_c4_chan_8way.jsonl, bench.py --config c4 --emulate r/8;
# residuals within 4 %):
#   * bucketing + gridding per channel (52.3 Mvis each), piecewise linear in
#     frequency (ms at 50, 110, ..., 350 MHz);
#   * 1.41 ms per resident w plane (zeroing, FFT, w-screen), the plane count
#     growing with the block's top frequency (w range ~ f_hi) -- the term that
#     limits strong scaling: at 8 ranks the planes are held 5x over;
#   * a batch of the stream costs no measurable extra beyond its channels;
#   * 2.7 ms fixed (plan, all-reduce excluded).
C4_CHAN_COST = ((50e6, 5.64), (110e6, 4.94), (170e6, 5.28), (230e6, 5.22), (290e6, 5.14),
                (350e6, 5.87))
C4_BATCH_MS = 0.0
C4_MAX_BATCH = 40
C4_PLANE_MS = 1.41
C4_FIXED_MS = 2.7
C4_PLANES = (0.179e-6, 8.33)  # nplanes ~ a f_hi + b


def c4_block_cost(freqs, max_batch=C4_MAX_BATCH):
    """Modelled invert time (ms) of one rank holding the channels `freqs`
    (one shared plane layout, one FFT pass, batches of <= max_batch)."""
    f = np.asarray(freqs, dtype=float)
    if f.size == 0:
        return 0.0
    xs, ys = zip(*C4_CHAN_COST)
    per_chan = float(np.interp(f, xs, ys).sum())
    batches = -(-f.size // max_batch)
    return (C4_FIXED_MS + per_chan + C4_BATCH_MS * (batches - 1) +
            C4_PLANE_MS * (C4_PLANES[0] * float(f.max()) + C4_PLANES[1]))


def balanced_channel_blocks(freqs, world, cost=c4_block_cost):
    """Contiguous channel blocks [(lo, hi)] for `world` ranks whose modelled
    costs are as equal as possible (minimise the maximum: bisection on the
    target with a greedy sweep).  Contiguous blocks keep each rank's w range
    (hence its plane count) small; the cost model moves channels from the
    high band, which carries the most w planes, to the low band."""
    n = len(freqs)
    if world <= 1:
        return [(0, n)]

    def sweep(target):
        blocks, lo = [], 0
        for r in range(world):
            hi = lo
            while hi < n and (hi == lo or cost(freqs[lo:hi + 1]) <= target) and \
                    n - (hi + 1) >= world - r - 1:
                hi += 1
            if r == world - 1:
                hi = n
            blocks.append((lo, hi))
            lo = hi
        return blocks

    lo_t, hi_t = 0.0, cost(freqs)
    for _ in range(60):
        mid = 0.5 * (lo_t + hi_t)
        b = sweep(mid)
        if max(cost(freqs[a:e]) for a, e in b) <= mid:
            hi_t = mid
        else:
            lo_t = mid
    return sweep(hi_t)


# w-slab partition of a band's invert (SDP_HIP_W_SLAB).  Every rank scans the
# whole band and grids only the visibilities whose first w plane lies in its
# contiguous slab of the band's plane layout, so it holds, transforms and
# screens only its slab's planes plus a W - 1 halo: the band's plane work is
# ~ nps + (world - 1)(W - 1) planes in total, not the sum over channel blocks
# of each block's own w range.  The image-domain sum of the slabs' images is
# the full image (each visibility is gridded once; the planes a slab holds
# are the footprints of its own visibilities).  Cost per rank (ms): gridding
# + bucketing per gridded visibility, the skip test per scanned visibility,
# per held plane (zeroing, FFT, w-screen), fixed.
WSLAB_VIS_MS_PER_G = 99.0    # C4 N = 1: (prep 619 + grid 709 ms) / 13.4 Gvis
WSLAB_SCAN_MS_PER_G = 4.0    # slab test of the visibilities of other slabs
WSLAB_PLANE_MS = 1.55        # C4 N = 1: (FFT 97 + screen 11 ms) / 71 planes, + zeroing
WSLAB_FIXED_MS = 4.2


def first_plane_histogram(uvw, freqs, layout, flip_uw=True):
    """Visibilities per first w plane of ``layout`` (kernels.wstack_layout) over
    the rows ``uvw`` [nrow, 3] (device, metres) and all ``freqs``: p0 =
    floor((w f / c - w0) / dw - W / 2) + 1, as the bucketing computes it."""
    w = uvw[:, 2].to(torch.float64) * (-1.0 if flip_uw else 1.0)
    nps, W, w0, dw = layout["nps"], layout["support"], layout["w0"], layout["dw"]
    hist = torch.zeros(nps, dtype=torch.float64, device=uvw.device)
    for f in np.asarray(freqs, dtype=float):
        pw = (w * (f / 299792458.0) - w0) / dw
        p0 = torch.floor(torch.clamp(pw - 0.5 * W, -2.0, 2.0e9)).to(torch.int64) + 1
        hist += torch.bincount(p0.clamp(0, nps - 1), minlength=nps)[:nps].to(torch.float64)
    return hist.cpu().numpy()


def wslab_cost(hist, lo, hi, W, nvis_total):
    """Modelled invert time (ms) of the rank holding first planes [lo, hi)."""
    n = float(np.sum(hist[lo:hi]))
    return (WSLAB_FIXED_MS + WSLAB_VIS_MS_PER_G * n / 1e9 +
            WSLAB_SCAN_MS_PER_G * (nvis_total - n) / 1e9 + WSLAB_PLANE_MS * (hi - lo + W - 1))


def wslab_partition(hist, world, W):
    """Contiguous first-plane slabs [(lo, hi)] covering [0, len(hist)) for
    `world` ranks, minimising the largest modelled cost (bisection on the
    target with a greedy sweep; every slab holds at least one first plane)."""
    nps = len(hist)
    nvis = float(np.sum(hist))
    if world <= 1 or nps <= 1:
        return [(0, nps)]
    world_eff = min(world, nps)

    def sweep(target):
        slabs, lo = [], 0
        for r in range(world_eff):
            hi = lo + 1
            while hi < nps and nps - hi > world_eff - r - 1 and \
                    wslab_cost(hist, lo, hi + 1, W, nvis) <= target:
                hi += 1
            if r == world_eff - 1:
                hi = nps
            slabs.append((lo, hi))
            lo = hi
        return slabs

    lo_t, hi_t = 0.0, wslab_cost(hist, 0, nps, W, nvis)
    for _ in range(60):
        mid = 0.5 * (lo_t + hi_t)
        sl = sweep(mid)
        if max(wslab_cost(hist, a, e, W, nvis) for a, e in sl) <= mid:
            hi_t = mid
        else:
            lo_t = mid
    slabs = sweep(hi_t)
    # more ranks than first planes: the extra ranks get empty slabs
    return slabs + [(nps, nps)] * (world - world_eff)


# Row partition by w (the default C4 strong-scaling partition): ranks own
# contiguous intervals of the rows' w (metres) and grid ALL channels of their
# rows, each with its own w-plane layout.  A row's w_lambda over the band is
# w f / c, so a rank of small-|w| rows holds few planes and a rank of
# large-|w| rows holds many but gets fewer rows: the cuts balance the cost
# below.  Plane work is ~2x the single-GPU planes in total at 8 ranks, not
# ~5x as with channel blocks (whose top-band block holds every plane), and no
# rank scans visibilities it does not grid (unlike the w-slab partition).
# Per-visibility cost (bucketing + gridding) grows with the row's |w| -- the
# long baselines fill sparse cells whose regions flush more atomics per
# record: (65.1 + 53.7 sqrt(|w| / max|w|)) ms per Gvis, a least-squares fit
# to the 8-way emulation (profiles/r03_c4_wrow_8way.jsonl, rms 6 ms/Gvis);
# planes 1.49 ms each.
WROW_VIS_MS_PER_G = 65.1
WROW_VIS_W_MS_PER_G = 53.7
WROW_PLANE_MS = 1.49
WROW_FIXED_MS = 3.0


def wrow_planes(wa, wb, f_lo, f_hi, dw, W):
    """Planes a rank holds whose rows' w (metres, sign applied) span [wa, wb]
    over frequencies [f_lo, f_hi]: its w_lambda range / dw plus the support."""
    c = 299792458.0
    lo = wa * (f_hi if wa < 0 else f_lo) / c
    hi = wb * (f_hi if wb > 0 else f_lo) / c
    return (hi - lo) / dw + W


def wrow_partition(w, freqs, world, dw, W, vis_ms_per_g=WROW_VIS_MS_PER_G,
                   vis_w_ms_per_g=WROW_VIS_W_MS_PER_G, plane_ms=WROW_PLANE_MS,
                   fixed_ms=WROW_FIXED_MS):
    """Contiguous w intervals of the rows for `world` ranks minimising the
    largest modelled cost (ms): the rows' channels x a vis cost rising with
    sqrt(|w| / max|w|) + held planes x plane cost + fixed (bisection on the
    target, greedy sweep with a binary search per rank).  ``w``: the rows' w in metres with the imaging sign
    convention applied (numpy).  Returns (order, cuts, costs): rank r owns
    rows order[cuts[r]:cuts[r + 1]]."""
    w = np.asarray(w, dtype=float)
    order = np.argsort(w, kind="stable")
    ws = w[order]
    n = ws.size
    f = np.asarray(freqs, dtype=float)
    f_lo, f_hi, nch = float(f.min()), float(f.max()), f.size
    wmax = float(np.max(np.abs(ws))) if n else 1.0
    # prefix sums of the per-row vis cost (ms)
    row_ms = (vis_ms_per_g + vis_w_ms_per_g * np.sqrt(np.abs(ws) / max(wmax, 1e-300))) * nch / 1e9
    pre = np.concatenate([[0.0], np.cumsum(row_ms)])

    def cost(i, j):
        if j <= i:
            return 0.0
        return (pre[j] - pre[i] +
                plane_ms * wrow_planes(ws[i], ws[j - 1], f_lo, f_hi, dw, W) + fixed_ms)

    if world <= 1 or n == 0:
        return order, [0, n], [cost(0, n)]

    def sweep(target):
        cuts, i = [0], 0
        for r in range(world):
            if i >= n:
                cuts.append(n)
                continue
            if r == world - 1:
                cuts.append(n)
                i = n
                continue
            a, b = i + 1, n
            if cost(i, a) > target:
                return None
            while a < b:
                m = (a + b + 1) // 2
                if cost(i, m) <= target:
                    a = m
                else:
                    b = m - 1
            cuts.append(a)
            i = a
        return cuts if cost(cuts[-2], n) <= target else None

    lo_t, hi_t = 0.0, cost(0, n)
    best = [0] * world + [n]
    for _ in range(60):
        mid = 0.5 * (lo_t + hi_t)
        c = sweep(mid)
        if c is not None:
            hi_t, best = mid, c
        else:
            lo_t = mid
    return order, best, [cost(a, e) for a, e in zip(best[:-1], best[1:])]


def invert_batched_shard(uvw, freq, vis_of_block, blocks, npix, cell, epsilon=1e-7,
                         do_wstacking=True, flip_uw=True, out=None, timer=None, bounds=None,
                         slab=None, batch_fn=None):
    """Invert one rank's channels as a sequence of channel blocks streamed
    through shared resident w planes (kernels.ms2dirty_batch: one plane
    layout from the merged bounds, one FFT pass).  ``vis_of_block(a, e)``
    returns the [nrow, e - a] device visibilities of channels a..e (generated
    or loaded on demand); ``timer`` (optional) is a context-manager factory
    wrapped around each device call so the caller can exclude the input
    staging from its timing.  Unit weights.  Returns the dirty image in
    RASCIL [y, x] order (unnormalised) accumulated into ``out``.  ``bounds``:
    the sequence's plane layout (default: merged over ``blocks``); ``slab`` =
    (lo, hi): a w-slab rank's first planes of that layout (wslab_partition),
    ``blocks`` then covering the whole band."""
    from . import kernels
    dev = uvw.device
    if out is None:
        out = torch.zeros((npix, npix), dtype=torch.float64, device=dev)
    if slab is not None and slab[0] >= slab[1]:
        return out  # (an empty slab: more ranks than first planes)
    b = bounds or kernels.merge_bounds(*[kernels.uvw_bounds(uvw, freq[a:e]) for a, e in blocks])
    fn = batch_fn or kernels.ms2dirty_batch
    for i, (a, e) in enumerate(blocks):
        vis = vis_of_block(a, e)
        ctx = timer() if timer else _nullctx()
        with ctx:
            fn(uvw, freq[a:e], vis, None, npix, npix, cell, cell, b,
                                   first=i == 0, last=i == len(blocks) - 1, epsilon=epsilon,
                                   do_wstacking=do_wstacking, flip_uw=flip_uw, out=out,
                                   out_strides=(1, npix), accumulate=True, slab=slab)
        del vis
    return out


def invert_wslab(uvw, freq, vis_of_block, blocks, npix, cell, epsilon=1e-7, do_wstacking=True,
                 flip_uw=True, bounds=None, group=None, out=None, timer=None, batch_fn=None):
    """w-slab multi-GPU invert of one band: every rank streams ALL the band's
    channel ``blocks`` (the SPMD form in which every rank holds the band, as
    the API sharding assumes) and grids only its slab of the band's first w
    planes (wslab_partition over first_plane_histogram: modelled cost
    balanced), then ONE all-reduce of the image sums the slabs.  Returns
    (image [y, x] unnormalised, slabs).  ``batch_fn`` replaces
    kernels.ms2dirty_batch (CPU tests inject the exact-sum oracle)."""
    from . import kernels
    rank, world = (dist.get_rank(group), dist.get_world_size(group)) if _dist_on() else (0, 1)
    b = bounds or kernels.merge_bounds(*[kernels.uvw_bounds(uvw, freq[a:e]) for a, e in blocks])
    lay = kernels.wstack_layout(b, npix, npix, cell, cell, epsilon, do_wstacking, flip_uw=flip_uw)
    hist = first_plane_histogram(uvw, freq.detach().cpu().numpy(), lay, flip_uw=flip_uw)
    slabs = wslab_partition(hist, world, lay["support"])
    out = invert_batched_shard(uvw, freq, vis_of_block, blocks, npix, cell, epsilon, do_wstacking,
                               flip_uw, out=out, timer=timer, bounds=b,
                               slab=slabs[rank] if world > 1 else None, batch_fn=batch_fn)
    if world > 1:
        all_reduce_sum(out, group)
    return out, slabs


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _gridder():
    from . import kernels
    return kernels.ms2dirty


def invert_sharded(uvw, freq, vis, wgt, npix, cell, epsilon=1e-7, do_wstacking=True,
                   flip_uw=True, normalise=True, group=None, grid_fn=None, out=None,
                   fused_sumwt=False):
    """Invert this rank's shard and all-reduce.

    uvw [nrow,3], freq [nchan_shard], vis/wgt [nrow, nchan_shard] are the
    rank-local arrays.  Returns (dirty [npix, npix] in RASCIL [y, x] order,
    sumwt) identical on every rank.  ``fused_sumwt``: the weight sum comes
    from the gridding call itself (``grid_fn(..., sumwt=t)`` adds it to a
    one-element f64 device tensor, as kernels.ms2dirty_vis's count pass does
    while it reads the weights) instead of a separate reduction over them.
    """
    grid_fn = grid_fn or _gridder()
    dev = uvw.device
    if out is None:
        out = torch.zeros((npix, npix), dtype=torch.float64, device=dev)
    else:
        out.zero_()
    extra = {}
    if fused_sumwt:
        extra["sumwt"] = torch.zeros(1, dtype=torch.float64, device=dev)
    if freq.numel() > 0 and uvw.shape[0] > 0:
        grid_fn(uvw, freq, vis, wgt, npix, npix, cell, cell, epsilon, do_wstacking,
                flip_uw=flip_uw, out=out, out_strides=(1, npix), accumulate=True, **extra)
    if fused_sumwt:
        sumwt = extra["sumwt"]
    else:
        sumwt = (wgt.sum() if wgt is not None else torch.tensor(float(vis.numel()), device=dev))
        sumwt = sumwt.to(torch.float64).reshape(1)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(sumwt, op=dist.ReduceOp.SUM, group=group)
    if normalise:
        # on the device (no host sync, so calls on two streams can overlap):
        # image / sumwt, or zeros when sumwt is 0 (normalise_sumwt)
        out.mul_(torch.where(sumwt > 0, 1.0 / sumwt, torch.zeros_like(sumwt)))
    return out, sumwt


def invert_wrow(uvw, freq, vis, wgt, npix, cell, epsilon=1e-7, do_wstacking=True, flip_uw=True,
                normalise=True, group=None, grid_fn=None, out=None, layout=None):
    """Row partition by w (wrow_partition): every rank holds the full [nrow,
    nchan] arrays (the SPMD form of the API sharding), grids ALL channels of
    its interval of the rows' w into its own w-plane layout, and one
    all-reduce of the image and sumwt combines the ranks.  ``layout``
    (support, dw) defaults to kernels.wstack_layout over the full band.
    Returns (dirty [y, x], sumwt, (order, cuts))."""
    from . import kernels
    rank, world = (dist.get_rank(group), dist.get_world_size(group)) if _dist_on() else (0, 1)
    if layout is None:
        b = kernels.uvw_bounds(uvw, freq)
        layout = kernels.wstack_layout(b, npix, npix, cell, cell, epsilon, do_wstacking,
                                       flip_uw=flip_uw)
    w = uvw[:, 2].detach().to("cpu", torch.float64).numpy() * (-1.0 if flip_uw else 1.0)
    order, cuts, _ = wrow_partition(w, freq.detach().cpu().numpy(), world, layout["dw"],
                                    layout["support"])
    rows = torch.as_tensor(order[cuts[rank]:cuts[rank + 1]], device=uvw.device)
    sub = lambda t: None if t is None else t[rows].contiguous()  # noqa: E731
    img, sw = invert_sharded(sub(uvw), freq, sub(vis), sub(wgt), npix, cell, epsilon,
                             do_wstacking, flip_uw, normalise, group, grid_fn, out)
    return img, sw, (order, cuts)


def _dist_on():
    return dist.is_available() and dist.is_initialized()


def _degridder():
    from . import kernels
    return kernels.dirty2ms


def predict_sharded(uvw, freq, model, cell, epsilon=1e-7, do_wstacking=True, flip_uw=True,
                    group=None, src=0, degrid_fn=None, vis_dtype=torch.complex64):
    """Channel-sharded predict (SURVEY.md §8(e) "predict: broadcast model,
    no exchange"; reference imaging/ng.py:38-143).

    ``model`` [npix, npix] f64 in RASCIL [y, x] order is broadcast from rank
    ``src`` (one npix^2 * 8 B broadcast); every rank then degrids its own
    channels ``freq`` for rows ``uvw``.  Returns the rank-local vis
    [nrow, nchan_shard].
    """
    degrid_fn = degrid_fn or _degridder()
    if _dist_on():
        dist.broadcast(model, src=src, group=group)
    npix = model.shape[-1]
    if freq.numel() == 0 or uvw.shape[0] == 0:
        return torch.zeros((uvw.shape[0], freq.numel()), dtype=vis_dtype, device=uvw.device)
    # the model is [y, x]: hand it to the ducc0-convention kernel as x-major
    vis, _ = degrid_fn(uvw, freq, model, None, cell, cell, epsilon, do_wstacking,
                       flip_uw=flip_uw, dirty_strides=(1, npix), npix=(npix, npix),
                       vis_dtype=vis_dtype)
    return vis


def dft_sharded(direction_cosines, fluxes, uvw, freq=None, group=None, src=0, dft_fn=None):
    """Row-sharded sky-component DFT (SURVEY.md §8(e) "DFT: shard rows,
    components replicated"; reference imaging/dft.py:32-182).  The component
    table is broadcast from rank ``src`` so every rank uses the same one; the
    rank's rows of ``uvw`` are predicted with no exchange."""
    if dft_fn is None:
        from . import kernels
        dft_fn = kernels.dft_point
    if _dist_on():
        dist.broadcast(direction_cosines, src=src, group=group)
        dist.broadcast(fluxes, src=src, group=group)
    return dft_fn(direction_cosines, fluxes, uvw, freq=freq)


def normalise_gains_global(gain, normalise_gains, group=None):
    """The reference's gain normalisation over the WHOLE table
    (calibration/solvers.py:135-143) when the gain rows are sharded:
    mean -> one all-reduce of (sum |g|, count); median -> all-gather of |g|
    (numpy median: mean of the two middle values for even counts)."""
    ga = gain.abs().flatten()
    if normalise_gains == "mean":
        acc = torch.stack([ga.sum(), torch.tensor(float(ga.numel()), dtype=ga.dtype,
                                                  device=ga.device)])
        if _dist_on():
            dist.all_reduce(acc, op=dist.ReduceOp.SUM, group=group)
        gabs = acc[0] / acc[1]
    elif normalise_gains == "median":
        if _dist_on():
            world = dist.get_world_size(group)
            n = torch.tensor([ga.numel()], device=ga.device)
            ns = [torch.zeros_like(n) for _ in range(world)]
            dist.all_gather(ns, n, group=group)
            nmax = int(max(int(x.item()) for x in ns))
            pad = torch.full((nmax,), float("nan"), dtype=ga.dtype, device=ga.device)
            pad[:ga.numel()] = ga
            parts = [torch.empty_like(pad) for _ in range(world)]
            dist.all_gather(parts, pad, group=group)
            allg = torch.cat([p[:int(k.item())] for p, k in zip(parts, ns)])
        else:
            allg = ga
        srt = torch.sort(allg).values
        m = srt.numel()
        gabs = 0.5 * (srt[(m - 1) // 2] + srt[m // 2])
    else:
        return gain
    return gain / gabs


def solve_gains_sharded(xb, wb, gain, gwt, row_start, ant2, mode, niter=200, tol=1e-6,
                        phase_only=True, normalise_gains=None, group=None, solve_fn=None):
    """Gain rows sharded across ranks (SURVEY.md §8(e) "solve_gaintable:
    embarrassingly parallel ... except the global normalise_gains").  Each
    rank solves its rows ``xb/wb/gain/gwt`` [rows_local, ...] with no
    collective, then the optional mean/median normalisation is global."""
    if solve_fn is None:
        from . import kernels
        solve_fn = kernels.solve_gains
    residual, used = solve_fn(xb, wb, gain, gwt, row_start, ant2, mode, niter=niter, tol=tol,
                              phase_only=phase_only)
    if normalise_gains in ("mean", "median") and not phase_only:
        gain.copy_(normalise_gains_global(gain, normalise_gains, group))
    return residual, used


def grid_cf_sharded(maps, vis_to_im, vis, wt, cf, grid, sumwt, group=None, grid_fn=None):
    """Row-sharded convolution-function gridding (SURVEY.md §8(e) "AW
    grid/degrid: one exchange step"; reference grid_data/gridding.py:160-255):
    each rank grids its rows into ``grid``/``sumwt`` (zeroed by the caller),
    then one all-reduce of the GridData and of sumwt."""
    if grid_fn is None:
        from . import kernels
        grid_fn = kernels.grid_cf
    grid_fn(maps, vis_to_im, vis, wt, cf, grid, sumwt)
    if _dist_on():
        dist.all_reduce(grid, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(sumwt, op=dist.ReduceOp.SUM, group=group)
    return grid, sumwt


def weight_sharded(uvw, freq, weight, flags, vis_to_im, wcs, grid, sumwt, imaging_weight,
                   weighting="uniform", robustness=0.0, group=None, grid_fn=None,
                   reweight_fn=None):
    """Channel-sharded weight_visibility (reference imaging/weighting.py:35-68
    with grid_data/gridding.py:258-499): each rank grids the flagged weights
    of its channels into ``grid``/``sumwt`` (zeroed by the caller), one
    all-reduce of the weight grid and of sumwt gives every rank the global
    grid, then each rank reweights its own samples with no further exchange.
    Robust weighting uses the all-reduced sumwt, as weight_visibility passes
    the gridding's sumwt.  Returns the rank-local imaging_weight."""
    if grid_fn is None or reweight_fn is None:
        from . import kernels
        grid_fn = grid_fn or kernels.grid_weights
        reweight_fn = reweight_fn or kernels.reweight
    if weighting != "natural":
        grid_fn(uvw, freq, weight, flags, vis_to_im, wcs, grid, sumwt)
        if _dist_on():
            dist.all_reduce(grid, op=dist.ReduceOp.SUM, group=group)
            dist.all_reduce(sumwt, op=dist.ReduceOp.SUM, group=group)
    return reweight_fn(uvw, freq, weight, flags, vis_to_im, wcs, grid, imaging_weight,
                       weighting=weighting, robustness=robustness, sumwt=sumwt)
