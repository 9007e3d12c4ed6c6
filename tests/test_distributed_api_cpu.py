"""CPU, world_size 2 over gloo: the reference-shaped API itself -- invert_ng
and predict_ng -- sharding a replicated Visibility across ranks when asked to
(shard=True) with torch.distributed initialised (imaging/ng.py: rows split into intervals
of w for an MFS invert, channel blocks from parallel.balanced_channel_blocks
otherwise; one all-reduce of image + sumwt for invert, an all-gather of the
channel blocks for predict).  Every rank must
return the unsharded result.

There is no GPU here, so inside the test processes the two HIP entry points
invert_ng / predict_ng call (kernels.ms2dirty_vis, kernels.dirty2ms_vis) are
replaced by the exact-sum oracle and the device by the CPU (test injection:
what is checked is the API's partitioning and collectives, which run
unchanged).  The GPU counterpart, through the real kernels, is
tests/test_gpu_parallel.py::test_api_sharding_two_ranks_one_gpu."""

import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import nufft_oracle as orc

FLIP = np.array([-1.0, 1.0, -1.0])
SEEN = set()  # visibility channels (frequencies) this process computed
ROWS = set()  # rows (their u) this process gridded


BATCHES = []  # (first, last) of every batched call this process made


def _oracle_ms2dirty_vis(uvw, freq, vis, pol, wgt, flags, coef, npix_x, npix_y, px, py,
                         epsilon=1e-7, do_wstacking=True, flip_uw=False, out=None,
                         out_strides=None, accumulate=False, sumwt=None, shift_lmn=None,
                         keep_buckets=False, reuse_buckets=False, precision=None, slot=0,
                         bounds=None, first=False, last=False):
    assert shift_lmn is None
    if bounds is not None:
        BATCHES.append((first, last))
    SEEN.update(freq.numpy().tolist())
    ROWS.update(np.round(uvw.numpy()[:, 0], 6).tolist())
    m = 1.0 - flags.numpy().astype(float)
    w = wgt.numpy() * m[..., pol]
    if vis is None:
        v = np.ones(w.shape, complex)
    elif coef is None:
        v = vis.numpy()[..., pol] * m[..., pol]
    else:
        v = sum(complex(c) * vis.numpy()[..., k] * m[..., k] for k, c in enumerate(coef))
    d = orc.ms2dirty_exact(uvw.numpy() * (FLIP if flip_uw else 1.0), freq.numpy(), v, w, npix_x,
                           npix_y, px, py, do_wstacking)
    assert tuple(out_strides) == (1, npix_x)  # RASCIL's [y, x] image
    out += torch.as_tensor(d.T)
    if sumwt is not None:
        sumwt += float(w.sum())
    return out, {}


def _oracle_dirty2ms_vis(uvw, freq, dirty, out, coef, px, py, epsilon=1e-7, do_wstacking=True,
                         flip_uw=False, dirty_strides=None, npix=None, accumulate=False,
                         shift_lmn=None, precision=None):
    assert shift_lmn is None and tuple(dirty_strides) == (1, npix[0])
    SEEN.update(freq.numpy().tolist())
    v = orc.dirty2ms_exact(uvw.numpy() * (FLIP if flip_uw else 1.0), freq.numpy(),
                           dirty.numpy().T, None, px, py, do_wstacking)
    coef = [1.0] + [0.0] * (out.shape[2] - 1) if coef is None else coef
    for k, c in enumerate(coef):
        val = torch.as_tensor(complex(c) * v).to(out.dtype)
        if accumulate:
            out[..., k] += val
        else:
            out[..., k] = val
    return out, {}


def _host_bounds(uvw, freq):
    return [float(uvw[:, 2].min()), float(uvw[:, 2].max()), float(uvw[:, 0].abs().max()),
            float(uvw[:, 1].abs().max()), float(freq.min()), float(freq.max())]


def _patch():
    from ska_sdp_func_python_amd import _device, kernels
    _device.device = lambda: torch.device("cpu")
    kernels.ms2dirty_vis = _oracle_ms2dirty_vis
    kernels.dirty2ms_vis = _oracle_dirty2ms_vis
    kernels.uvw_bounds = _host_bounds


def _case(kind, seed=51):
    from ska_sdp_func_python_amd import datamodels as dm
    from gpu_helpers import vis_from_arrays
    rng = np.random.default_rng(seed)
    nt, nb, nchan = 3, 12, 5
    freq = np.linspace(1.0e9, 1.2e9, nchan)
    umax = 1200.0
    uvw = rng.uniform(-1, 1, (nt, nb, 3)) * umax * orc.C_LIGHT / freq.max()
    shape = (nt, nb, nchan, 1)
    v = rng.normal(size=shape) + 1j * rng.normal(size=shape)
    fl = (rng.uniform(size=shape) < 0.1).astype(int)
    vis = vis_from_arrays(uvw, freq, v, flags=fl, phasecentre=dm.SkyCoord(0.0, -0.6))
    vis["imaging_weight"] = rng.uniform(0.5, 2.0, shape)
    cube = kind == "invert_cube"
    fc, bw = (float(freq[0]), float(freq[1] - freq[0])) if cube else (float(freq.mean()), 1e9)
    if kind == "invert_mfsnarrow":  # an MFS image whose WCS maps no vis channel to 0
        bw = 1e6
    im = dm.create_image(32, 0.4 / umax, dm.SkyCoord(0.0, -0.6), frequency=fc,
                         channel_bandwidth=bw, nchan=nchan if cube else 1)
    if kind == "predict":
        im["pixels"].data[...] = rng.normal(size=im["pixels"].data.shape)
    return vis, im


def _run(kind, seed=51, **kw):
    from ska_sdp_func_python_amd.imaging import invert_ng, predict_ng
    vis, im = _case(kind, seed)
    if kind == "predict":
        return (np.asarray(predict_ng(vis, im, **kw).vis.data),)
    d, sw = invert_ng(vis, im, normalise=True, **kw)
    return np.asarray(d["pixels"].data), np.asarray(sw)


def _worker(rank, world, port, kind, q, shard=True, own_data=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _patch()
    try:
        kw = {} if shard is None else {"shard": shard}
        try:
            out = _run(kind, 51 + (rank if own_data else 0), **kw)
        except ValueError as e:
            out = ("ValueError", str(e))
        q.put((rank, out, sorted(SEEN), sorted(ROWS)))
    finally:
        dist.destroy_process_group()


def _spawn(kind, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + int(np.random.default_rng().integers(0, 300))
    procs = [ctx.Process(target=_worker, args=(r, 2, port, kind, q), kwargs=kw) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert len(res) == 2
    return res


@pytest.mark.parametrize("kind", ["invert_mfs", "invert_cube", "predict"])
def test_reference_api_shards_across_ranks(kind, monkeypatch):
    from ska_sdp_func_python_amd import _device, kernels
    monkeypatch.setattr(_device, "device", lambda: torch.device("cpu"))
    monkeypatch.setattr(kernels, "ms2dirty_vis", _oracle_ms2dirty_vis)
    monkeypatch.setattr(kernels, "dirty2ms_vis", _oracle_dirty2ms_vis)
    ref = _run(kind)  # this process: no process group, so unsharded
    res = _spawn(kind, shard=True)
    if kind == "invert_mfs":
        # an MFS w-stacked invert splits the rows (intervals of w, all channels)
        rows = [set(r) for _, _, _, r in res]
        assert rows[0] and rows[1] and not (rows[0] & rows[1]) and len(rows[0] | rows[1]) == 36
    else:
        # the ranks computed disjoint channel blocks that cover the band
        seen = [set(s) for _, _, s, _ in res]
        assert seen[0] and seen[1] and not (seen[0] & seen[1]) and len(seen[0] | seen[1]) == 5
    for _, out, _, _ in res:
        for a, b in zip(out, ref):
            np.testing.assert_allclose(a, b, rtol=1e-10, atol=1e-12)


def test_default_is_per_rank_and_mismatched_shards_raise(monkeypatch):
    """Without shard=True every rank computes its own call (a data-parallel
    pipeline passes each rank its own data, as with the reference); with
    shard=True ranks that pass different data get ValueError on every rank
    instead of an image combined from unrelated partial results."""
    from ska_sdp_func_python_amd import _device, kernels
    monkeypatch.setattr(_device, "device", lambda: torch.device("cpu"))
    monkeypatch.setattr(kernels, "ms2dirty_vis", _oracle_ms2dirty_vis)
    monkeypatch.setattr(kernels, "dirty2ms_vis", _oracle_dirty2ms_vis)
    refs = [_run("invert_mfs", 51 + r) for r in range(2)]
    res = _spawn("invert_mfs", shard=None, own_data=True)
    for rank, out, _, rows in res:
        assert len(rows) == 36  # every row of its own observation
        for a, b in zip(out, refs[rank]):
            np.testing.assert_allclose(a, b, rtol=1e-10, atol=1e-12)
    res = _spawn("invert_mfs", shard=True, own_data=True)
    for _, out, _, _ in res:
        assert out[0] == "ValueError" and "same inputs" in out[1]


def _check_worker(rank, world, port, q, own):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ska_sdp_func_python_amd import parallel
    try:
        rng = np.random.default_rng(5 + (rank if own else 0))
        vis = (rng.normal(size=(40, 3, 2)) + 1j * rng.normal(size=(40, 3, 2))).astype(np.complex64)
        vis[::7, 1, 0] = np.nan  # flagged NaN samples, replicated on every rank
        wgt = torch.as_tensor(rng.uniform(size=(40, 3)))
        wgt[3, 2] = float("nan")
        flags = np.zeros((40, 3, 2), np.int8)
        try:
            parallel.check_replicated((rank, world, None), [vis, wgt, flags, (4, 1, 32, 32)],
                                      "invert_ng")
            q.put((rank, "ok"))
        except ValueError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("own", [False, True])
def test_replication_check_is_bitwise_and_nan_safe(own):
    """parallel.check_replicated hashes the inputs' bytes in chunks (no
    float64 copy of the Visibility): replicated inputs holding NaNs pass on
    every rank; ranks with different data raise ValueError on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + int(np.random.default_rng().integers(300, 600))
    procs = [ctx.Process(target=_check_worker, args=(r, 2, port, q, own)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for _, msg in res:
        if own:
            assert "same inputs" in msg
        else:
            assert msg == "ok"


def test_byte_hash_matches_between_host_and_torch():
    """The hash of an array is the same whether a rank holds it as numpy or
    as a torch tensor, and whatever the chunking."""
    from ska_sdp_func_python_amd import parallel
    rng = np.random.default_rng(3)
    for a in (rng.normal(size=1001), (rng.normal(size=(17, 3)) + 1j).astype(np.complex64),
              rng.integers(0, 2, (33, 5)).astype(np.int8), np.array([np.nan, 1.0, -0.0])):
        h = parallel._byte_hash(a)
        assert h == parallel._byte_hash(torch.as_tensor(a))
        old = parallel._HASH_CHUNK
        try:
            parallel._HASH_CHUNK = 24
            assert parallel._byte_hash(a) == h == parallel._byte_hash(torch.as_tensor(a))
        finally:
            parallel._HASH_CHUNK = old
    assert parallel._byte_hash(np.array([1.0, 2.0])) != parallel._byte_hash(np.array([2.0, 1.0]))


def _local_worker(rank, world, port, kind, q, max_call=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if max_call:
        os.environ["SDP_HIP_MAX_CALL_GVIS"] = max_call
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _patch()
    try:
        q.put((rank, _run_local(kind, rank, world), sorted(SEEN), sorted(ROWS), list(BATCHES)))
    finally:
        dist.destroy_process_group()


def _block(vis, rank, world, by):
    """This rank's own Visibility: its time rows or its channels."""
    from gpu_helpers import vis_from_arrays
    nt, _, nchan, _ = vis.vis.data.shape
    t = slice(rank * nt // world, (rank + 1) * nt // world) if by == "rows" else slice(0, nt)
    c = slice(rank * nchan // world, (rank + 1) * nchan // world) if by == "chans" else slice(0, nchan)
    if by == "chans1":  # rank 0 holds a single channel of the band
        c = slice(0, 1) if rank == 0 else slice(1, nchan)
    b = vis_from_arrays(np.asarray(vis.uvw.data)[t], np.asarray(vis.frequency.data)[c],
                        np.asarray(vis.vis.data)[t, :, c], weight=np.asarray(vis.weight.data)[t, :, c],
                        flags=np.asarray(vis.flags.data)[t, :, c], phasecentre=vis.phasecentre)
    b["imaging_weight"] = np.asarray(vis.imaging_weight.data)[t, :, c]
    return b, t, c


def _run_local(kind, rank, world):
    from ska_sdp_func_python_amd.imaging import invert_ng, predict_ng
    base = {"invert_rows": "invert_mfs", "invert_chans": "invert_cube", "predict_chans": "predict",
            "invert_chans1": "invert_mfsnarrow", "invert_rowseps": "invert_mfs"}
    vis, im = _case(base[kind])
    mine, t, c = _block(vis, rank, world, kind.split("_")[1].replace("rowseps", "rows"))
    if kind == "predict_chans":
        return np.asarray(predict_ng(mine, im, shard="local").vis.data), (t.start, t.stop, c.start, c.stop)
    kw = {}
    if kind == "invert_rowseps":  # the ranks disagree on epsilon: refused on both
        kw["epsilon"] = 1e-12 if rank == 0 else 1e-6
        try:
            invert_ng(mine, im, normalise=True, shard="local", **kw)
        except ValueError as e:
            return ("ValueError", str(e))
        return ("no error",)
    d, sw = invert_ng(mine, im, normalise=True, shard="local")
    return np.asarray(d["pixels"].data), np.asarray(sw)


def test_presharded_local_mode_refuses_mismatched_options():
    """shard="local" checks the call's scalar options across the ranks as
    well as the image geometry: ranks passing different epsilon would
    otherwise all-reduce images of different precision."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + int(np.random.default_rng().integers(300, 590))
    procs = [ctx.Process(target=_local_worker, args=(r, 2, port, "invert_rowseps", q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for _, out, *_ in res:
        assert out[0] == "ValueError" and "same inputs" in out[1]


@pytest.mark.parametrize("kind", ["invert_rows", "invert_chans", "invert_chans1", "predict_chans"])
@pytest.mark.parametrize("max_call", [None, "1e-8"])
def test_presharded_local_mode(kind, max_call, monkeypatch):
    """shard="local": each rank passes its OWN block of the observation (its
    time rows, or its channels); invert_ng all-reduces the partial images
    and weight sums, so both ranks return the whole observation's image;
    predict_ng predicts each block with no exchange.  With
    SDP_HIP_MAX_CALL_GVIS tiny, the rank's calls run as channel-batch
    sequences (first ... last) through sdp_hip_ms2dirty_vis_batch."""
    from ska_sdp_func_python_amd import _device, kernels
    monkeypatch.setattr(_device, "device", lambda: torch.device("cpu"))
    monkeypatch.setattr(kernels, "ms2dirty_vis", _oracle_ms2dirty_vis)
    monkeypatch.setattr(kernels, "dirty2ms_vis", _oracle_dirty2ms_vis)
    ref = _run({"invert_rows": "invert_mfs", "invert_chans": "invert_cube",
                "invert_chans1": "invert_mfsnarrow", "predict_chans": "predict"}[kind])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + int(np.random.default_rng().integers(600, 900))
    procs = [ctx.Process(target=_local_worker, args=(r, 2, port, kind, q, max_call))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, out, seen, rows, batches in res:
        if max_call and kind == "invert_rows":  # (the cube: one channel per call)
            assert batches and batches[0] == (True, False) and batches[-1] == (False, True)
        if kind == "predict_chans":
            t0, t1, c0, c1 = out[1]
            np.testing.assert_allclose(out[0], ref[0][t0:t1, :, c0:c1], rtol=1e-10, atol=1e-12)
        else:
            for a, b in zip(out, ref):
                np.testing.assert_allclose(a, b, rtol=1e-10, atol=1e-12)
