"""CPU, world_size 2 over gloo: the channel-sharded invert + all-reduce equals
the unsharded invert.  The per-shard gridder is the exact-DFT oracle (test
injection), so this checks partitioning, reduction and normalisation."""

import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import nufft_oracle as orc


def _oracle_grid(uvw, freq, vis, wgt, nx, ny, px, py, eps, dow, flip_uw, out, out_strides,
                 accumulate):
    fl = np.array([-1.0, 1.0, -1.0]) if flip_uw else np.ones(3)
    d = orc.ms2dirty_exact(uvw.numpy() * fl, freq.numpy(), vis.numpy(), wgt.numpy(), nx, ny, px,
                           py, dow)
    out += torch.as_tensor(d.T)  # [y, x]
    return out, {}


def _worker(rank, world, port, data, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ska_sdp_func_python_amd.parallel import interleaved_channels, invert_sharded
    uvw, freq, vis, wgt, npix, cell = data
    ch = interleaved_channels(len(freq), rank, world)
    img, sw = invert_sharded(torch.as_tensor(uvw), torch.as_tensor(freq[ch]),
                             torch.as_tensor(vis[:, ch]), torch.as_tensor(wgt[:, ch]), npix, cell,
                             grid_fn=_oracle_grid)
    q.put((rank, img.numpy(), float(sw.item())))
    dist.destroy_process_group()


def test_sharded_invert_equals_full():
    rng = np.random.default_rng(4)
    nrow, nchan, npix = 60, 5, 32
    freq = np.linspace(1e9, 1.2e9, nchan)
    uvw = rng.uniform(-1, 1, (nrow, 3)) * 1500 * 299792458.0 / freq.max()
    vis = rng.normal(size=(nrow, nchan)) + 1j * rng.normal(size=(nrow, nchan))
    wgt = rng.uniform(0.5, 1.5, (nrow, nchan))
    cell = 0.25 / 1500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + int(rng.integers(0, 500))
    procs = [ctx.Process(target=_worker, args=(r, 2, port, (uvw, freq, vis, wgt, npix, cell), q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    full = orc.ms2dirty_exact(uvw * np.array([-1.0, 1.0, -1.0]), freq, vis, wgt, npix, npix, cell,
                              cell, True).T / wgt.sum()
    for _, img, sw in res:
        np.testing.assert_allclose(sw, wgt.sum(), rtol=1e-12)
        np.testing.assert_allclose(img, full, rtol=1e-10, atol=1e-12)


# ---------------------------------------------------------------------------
# predict / DFT / StefCal / CF gridding shards; the compute
# is the oracle (test injection), the partitioning and collectives are the
# product's parallel.py
# ---------------------------------------------------------------------------
import ref_oracle as ro  # noqa: E402

FLIP = np.array([-1.0, 1.0, -1.0])


def _oracle_degrid(uvw, freq, dirty, wgt, px, py, eps, dow, flip_uw, dirty_strides, npix,
                   vis_dtype):
    img = dirty.numpy()
    if tuple(dirty_strides) == (1, npix[0]):  # [y, x] storage
        img = img.T
    v = orc.dirty2ms_exact(uvw.numpy() * (FLIP if flip_uw else 1.0), freq.numpy(), img, None, px,
                           py, dow)
    return torch.as_tensor(v), {}


def _oracle_dft(dc, fl, uvw, freq=None):
    uvwl = uvw.numpy()[:, None, :] * (freq.numpy() / 299792458.0)[None, :, None]
    return torch.as_tensor(ro.dft_cpu_looped(dc.numpy(), uvwl, fl.numpy()))


def _pairs(row_start, ant2):
    a1 = np.repeat(np.arange(len(row_start) - 1), np.diff(row_start))
    return np.stack([a1, np.asarray(ant2)], 1)


def _oracle_solve(xb, wb, gain, gwt, row_start, ant2, mode, niter=200, tol=1e-6,
                  phase_only=True):
    bl = _pairs(row_start, ant2)
    nants = gain.shape[1]
    res = []
    for s in range(xb.shape[0]):
        g0 = gain[s].numpy()
        g, w, r, _ = ro.stefcal_row(xb[s].numpy().copy(), wb[s].numpy().copy(), bl, nants, g0,
                                    gwt[s].numpy(), niter, tol, phase_only)
        gain[s] = torch.as_tensor(np.asarray(g).reshape(g0.shape))
        res.append(r)
    return torch.as_tensor(np.array(res)), None


def _oracle_grid_cf(maps, vis_to_im, vis, wt, cf, grid, sumwt):
    g, s = ro.grid_cf({k: v.numpy() for k, v in maps.items()}, vis_to_im.numpy(), vis.numpy(),
                      wt.numpy(), cf.numpy(), tuple(grid.shape))
    grid += torch.as_tensor(g)
    sumwt += torch.as_tensor(s)


def _shard_worker(rank, world, port, kind, data, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ska_sdp_func_python_amd import parallel as par
    T = torch.as_tensor
    if kind == "predict":
        uvw, freq, model, cell = data
        ch = par.interleaved_channels(len(freq), rank, world)
        m = T(model.copy()) if rank == 0 else torch.zeros_like(T(model))  # broadcast from 0
        out = par.predict_sharded(T(uvw), T(freq[ch]), m, cell, degrid_fn=_oracle_degrid)
        q.put((rank, ch, out.numpy()))
    elif kind == "dft":
        dc, fl, uvw, freq = data
        lo, hi = par.shard_range(uvw.shape[0], rank, world)
        dcs = T(dc.copy()) if rank == 0 else torch.zeros_like(T(dc))
        fls = T(fl.copy()) if rank == 0 else torch.zeros_like(T(fl))
        out = par.dft_sharded(dcs, fls, T(uvw[lo:hi]), T(freq), dft_fn=_oracle_dft)
        q.put((rank, (lo, hi), out.numpy()))
    elif kind == "solve":
        xb, wb, gain, gwt, rs, a2, norm = data
        lo, hi = par.shard_range(xb.shape[0], rank, world)
        g = T(gain[lo:hi].copy())
        par.solve_gains_sharded(T(xb[lo:hi]), T(wb[lo:hi]), g, T(gwt[lo:hi].copy()), rs, a2, 0,
                                phase_only=False, normalise_gains=norm, solve_fn=_oracle_solve)
        q.put((rank, (lo, hi), g.numpy()))
    elif kind == "cf":
        maps, v2i, vis, wt, cf, gshape = data
        lo, hi = par.shard_range(vis.shape[0], rank, world)
        grid = torch.zeros(gshape, dtype=torch.complex128)
        sumwt = torch.zeros(gshape[:2], dtype=torch.float64)
        mp_ = {k: T(v[:, lo:hi]) for k, v in maps.items()}
        par.grid_cf_sharded(mp_, T(v2i), T(vis[lo:hi]), T(wt[lo:hi]), T(cf), grid, sumwt,
                            grid_fn=_oracle_grid_cf)
        q.put((rank, None, (grid.numpy(), sumwt.numpy())))
    dist.destroy_process_group()


def _run(kind, data, seed):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30000 + seed * 7 + int(np.random.default_rng(seed).integers(0, 400))
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, kind, data, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    return res


def test_sharded_predict_equals_full():
    rng = np.random.default_rng(11)
    nrow, nchan, npix = 40, 4, 24
    freq = np.linspace(1e9, 1.2e9, nchan)
    uvw = rng.uniform(-1, 1, (nrow, 3)) * 800 * 299792458.0 / freq.max()
    model = rng.normal(size=(npix, npix))  # [y, x]
    cell = 0.25 / 800
    res = _run("predict", (uvw, freq, model, cell), 1)
    full = orc.dirty2ms_exact(uvw * FLIP, freq, model.T, None, cell, cell, True)
    for _, ch, v in res:
        np.testing.assert_allclose(v, full[:, ch], rtol=1e-10, atol=1e-12)


def test_sharded_dft_equals_full():
    rng = np.random.default_rng(12)
    nrow, ncomp = 30, 5
    freq = np.array([1.0e9, 1.1e9])
    uvw = rng.normal(0, 2000, (nrow, 3))
    lm = rng.uniform(-0.02, 0.02, (ncomp, 2))
    dc = np.concatenate([lm, (np.sqrt(1 - (lm ** 2).sum(1)) - 1)[:, None]], 1)
    fl = (rng.uniform(0.5, 2, (ncomp, 1, 1)) + 0j)
    res = _run("dft", (dc, fl, uvw, freq), 2)
    full = ro.dft_cpu_looped(dc, uvw[:, None, :] * (freq / 299792458.0)[None, :, None], fl)
    for _, (lo, hi), v in res:
        np.testing.assert_allclose(v, full[lo:hi], rtol=1e-12)


@pytest.mark.parametrize("norm", ["mean", "median"])
def test_sharded_solve_global_normalisation(norm):
    rng = np.random.default_rng(13)
    nants, nrows, nchan = 6, 3, 2
    a1, a2 = np.triu_indices(nants, 1)
    g = rng.lognormal(0, 0.2, (nrows, nants, nchan)) * np.exp(1j * rng.normal(0, 0.3, (nrows, nants, nchan)))
    xb = (g[:, a1] * np.conj(g[:, a2]))[..., None]
    wb = np.ones(xb.shape)
    rs = np.concatenate([[0], np.cumsum(np.bincount(a1, minlength=nants))]).astype(np.int32)
    gain = np.ones((nrows, nants, nchan, 1, 1), complex)
    gwt = np.zeros(gain.shape)
    res = _run("solve", (xb, wb, gain, gwt, rs, a2.astype(np.int32), norm), 3 + len(norm))
    # unsharded reference: all rows, then the same global normalisation
    gfull = torch.as_tensor(gain.copy())
    _oracle_solve(torch.as_tensor(xb), torch.as_tensor(wb), gfull, torch.as_tensor(gwt.copy()), rs,
                  a2, 0, phase_only=False)
    ga = np.abs(gfull.numpy())
    gfull = gfull.numpy() / (np.median(ga) if norm == "median" else np.mean(ga))
    for _, (lo, hi), gs in res:
        np.testing.assert_allclose(gs, gfull[lo:hi], rtol=1e-10, atol=1e-12)


def test_sharded_cf_gridding_equals_full():
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "cfgrid_p4.npz"))
    rng = np.random.default_rng(14)
    nrow, nchan, npol = 20, 1, 4
    ny = nx = 48
    maps = {k: rng.integers(lo, hi, (nchan, nrow)).astype(np.int32)
            for k, lo, hi in (("pu", 4, 44), ("pv", 4, 44), ("pwc", 0, 3), ("pdu", 0, 5),
                              ("pdv", 0, 5))}
    v2i = np.zeros(nchan, np.int32)
    vis = rng.normal(size=(nrow, nchan, npol)) + 1j * rng.normal(size=(nrow, nchan, npol))
    wt = rng.uniform(0.5, 1.5, (nrow, nchan, npol))
    cf = g["cf"]
    gshape = (1, npol, ny, nx)
    res = _run("cf", (maps, v2i, vis, wt, cf, gshape), 5)
    full, sw = ro.grid_cf(maps, v2i, vis, wt, cf, gshape)
    for _, _, (grid, sumwt) in res:
        np.testing.assert_allclose(grid, full, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(sumwt, sw, rtol=1e-12)


def _oracle_grid_weights(uvw, freq, weight, flags, v2i, wcs, grid, sumwt):
    import weighting_oracle as wo
    fw = (weight * (1 - flags)).numpy()
    g, s, _ = wo.grid_weights(uvw.numpy(), freq.numpy(), fw, v2i.numpy(), wcs, grid.shape[0],
                              grid.shape[2], grid.shape[3])
    grid += torch.as_tensor(g)
    sumwt += torch.as_tensor(s)


def _oracle_reweight(uvw, freq, weight, flags, v2i, wcs, grid, imaging_weight, weighting,
                     robustness, sumwt):
    import weighting_oracle as wo
    m = (1 - flags).numpy()
    out = wo.reweight(uvw.numpy(), freq.numpy(), weight.numpy() * m,
                      imaging_weight.numpy() * m, v2i.numpy(), wcs, grid.numpy(), weighting,
                      robustness, sumwt.numpy())
    imaging_weight.copy_(torch.as_tensor(out))
    return imaging_weight


def _weight_worker(rank, world, port, data, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ska_sdp_func_python_amd.parallel import interleaved_channels, weight_sharded
    uvw, freq, wt, flags, imw, wcs, n, weighting = data
    ch = interleaved_channels(len(freq), rank, world)
    grid = torch.zeros((1, 1, n, n), dtype=torch.float64)
    sumwt = torch.zeros((1, 1), dtype=torch.float64)
    out = weight_sharded(torch.as_tensor(uvw), torch.as_tensor(freq[ch]),
                         torch.as_tensor(wt[:, ch].copy()), torch.as_tensor(flags[:, ch].copy()),
                         torch.zeros(len(ch), dtype=torch.int32), wcs, grid, sumwt,
                         torch.as_tensor(imw[:, ch].copy()), weighting=weighting, robustness=0.5,
                         grid_fn=_oracle_grid_weights, reweight_fn=_oracle_reweight)
    q.put((rank, ch, out.numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("weighting", ["uniform", "robust"])
def test_sharded_weighting_equals_full(weighting):
    import weighting_oracle as wo
    rng = np.random.default_rng(8)
    nrow, nchan, n = 300, 6, 32
    freq = np.linspace(1e9, 1.2e9, nchan)
    uvw = rng.normal(size=(nrow, 3)) * 300.0
    wt = rng.uniform(0.5, 2.0, (nrow, nchan, 1))
    flags = (rng.uniform(size=(nrow, nchan, 1)) < 0.1).astype(np.int64)
    imw = rng.uniform(0.5, 2.0, (nrow, nchan, 1))
    du = 2 * np.abs(uvw[:, :2]).max() * freq.max() / wo.C_M_S / n
    wcs = ((0.0, -du, n // 2 + 1), (0.0, du, n // 2 + 1))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + int(rng.integers(500, 1000))
    args = (uvw, freq, wt, flags, imw, wcs, n, weighting)
    procs = [ctx.Process(target=_weight_worker, args=(r, 2, port, args, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    fw = wt * (1 - flags)
    v2i = np.zeros(nchan, int)
    grid, sumwt, _ = wo.grid_weights(uvw, freq, fw, v2i, wcs, 1, n, n)
    full = wo.reweight(uvw, freq, fw, imw * (1 - flags), v2i, wcs, grid, weighting, 0.5, sumwt)
    for _, ch, out in res:
        np.testing.assert_allclose(out, full[:, ch], rtol=1e-12)


# ---------------------------------------------------------------------------
# w-slab partition (parallel.invert_wslab): each rank grids only the
# visibilities whose first w plane of the band's layout lies in its slab; the
# per-slab gridder is the exact-sum oracle restricted to that slab (test
# injection), the layout query, histogram, partition and all-reduce are the
# product's
# ---------------------------------------------------------------------------
def _oracle_slab_batch(uvw, freq, vis, wgt, nx, ny, px, py, bounds, first, last, epsilon,
                       do_wstacking, flip_uw, out, out_strides, accumulate, slab):
    from ska_sdp_func_python_amd import kernels
    lay = kernels.wstack_layout(bounds, nx, ny, px, py, epsilon, do_wstacking, flip_uw=flip_uw)
    u = uvw.numpy() * (FLIP if flip_uw else 1.0)
    f = freq.numpy()
    v = vis.numpy() if vis is not None else np.ones((u.shape[0], f.size), complex)
    W = lay["support"]
    pw = (u[:, 2:3] * f[None, :] / 299792458.0 - lay["w0"]) / lay["dw"]
    p0 = np.floor(np.clip(pw - 0.5 * W, -2, 2e9)).astype(int) + 1
    lo, hi = slab if slab is not None else (0, lay["nps"])
    keep = ((p0 >= lo) & (p0 < hi)).astype(float)
    wt = (wgt.numpy() if wgt is not None else np.ones(v.shape)) * keep
    d = orc.ms2dirty_exact(u, f, v, wt, nx, ny, px, py, do_wstacking)
    out += torch.as_tensor(d.T)  # [y, x]
    return (out if last else None), {"nvis_used": int(keep.sum())}


def _wslab_worker(rank, world, port, data, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ska_sdp_func_python_amd.parallel import invert_wslab
    uvw, freq, vis, npix, cell, bounds = data
    V = torch.as_tensor(vis)
    img, slabs = invert_wslab(torch.as_tensor(uvw), torch.as_tensor(freq),
                              lambda a, e: V[:, a:e], [(0, 2), (2, len(freq))], npix, cell,
                              bounds=bounds, batch_fn=_oracle_slab_batch)
    q.put((rank, img.numpy(), slabs))
    dist.destroy_process_group()


def test_wslab_invert_two_ranks_equals_full():
    rng = np.random.default_rng(9)
    nrow, nchan, npix = 80, 4, 32
    freq = np.linspace(1e9, 1.3e9, nchan)
    uvw = rng.uniform(-1, 1, (nrow, 3)) * 1500 * 299792458.0 / freq.max()
    uvw[:, 2] *= 40.0  # many w planes
    vis = rng.normal(size=(nrow, nchan)) + 1j * rng.normal(size=(nrow, nchan))
    cell = 0.25 / 1500
    bounds = [uvw[:, 2].min(), uvw[:, 2].max(), np.abs(uvw[:, 0]).max(), np.abs(uvw[:, 1]).max(),
              freq.min(), freq.max()]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + int(rng.integers(500, 1000))
    procs = [ctx.Process(target=_wslab_worker, args=(r, 2, port, (uvw, freq, vis, npix, cell,
                                                                   bounds), q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    full = orc.ms2dirty_exact(uvw * FLIP, freq, vis, np.ones(vis.shape), npix, npix, cell, cell,
                              True).T
    for _, img, slabs in res:
        assert len(slabs) == 2 and slabs[0][0] == 0 and slabs[0][1] == slabs[1][0] < slabs[1][1]
        np.testing.assert_allclose(img, full, rtol=1e-10, atol=1e-12)


# ---------------------------------------------------------------------------
# row partition by w (parallel.invert_wrow): each rank grids all channels of
# its interval of the rows' w; the per-rank gridder is the exact-sum oracle
# (test injection), the partition and the all-reduces are the product's
# ---------------------------------------------------------------------------
def _wrow_worker(rank, world, port, data, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ska_sdp_func_python_amd.parallel import invert_wrow
    uvw, freq, vis, wgt, npix, cell = data
    img, sw, (order, cuts) = invert_wrow(torch.as_tensor(uvw), torch.as_tensor(freq),
                                         torch.as_tensor(vis), torch.as_tensor(wgt), npix, cell,
                                         grid_fn=_oracle_grid, layout={"dw": 40.0, "support": 8})
    q.put((rank, img.numpy(), float(sw.item()), cuts))
    dist.destroy_process_group()


def test_wrow_invert_two_ranks_equals_full():
    rng = np.random.default_rng(11)
    nrow, nchan, npix = 70, 4, 32
    freq = np.linspace(1e9, 1.3e9, nchan)
    uvw = rng.uniform(-1, 1, (nrow, 3)) * 1500 * 299792458.0 / freq.max()
    vis = rng.normal(size=(nrow, nchan)) + 1j * rng.normal(size=(nrow, nchan))
    wgt = rng.uniform(0.5, 1.5, (nrow, nchan))
    cell = 0.25 / 1500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + int(rng.integers(1000, 1500))
    procs = [ctx.Process(target=_wrow_worker, args=(r, 2, port, (uvw, freq, vis, wgt, npix, cell),
                                                    q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    full = orc.ms2dirty_exact(uvw * FLIP, freq, vis, wgt, npix, npix, cell, cell, True).T / wgt.sum()
    for _, img, sw, cuts in res:
        assert cuts[0] == 0 and cuts[-1] == nrow and 0 < cuts[1] < nrow
        np.testing.assert_allclose(sw, wgt.sum(), rtol=1e-12)
        np.testing.assert_allclose(img, full, rtol=1e-10, atol=1e-12)
