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
