"""Dev probe: does a spatially sorted visibility order speed up the CF
gridder's fp64 atomics?  The bench_paths cfgrid case (4 Mvis uniform over a
4096^2 grid, 8x8 taps), gridded in the given order and after sorting the
rows by (pv / T, pu / T) tile for a few tile sizes T."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
import numpy as np, torch
from ska_sdp_func_python_amd import kernels

dev = torch.device("cuda:0")
rng = np.random.default_rng(5)
nrow, nchan, npol = 4_000_000, 1, 1
ny = nx = 4096
gv = gu = 8
nw, ndv, ndu = 5, 8, 8
maps_h = {"pu": rng.integers(gu, nx - gu, (nchan, nrow)), "pv": rng.integers(gv, ny - gv, (nchan, nrow)),
          "pwc": rng.integers(0, nw, (nchan, nrow)), "pdu": rng.integers(0, ndu, (nchan, nrow)),
          "pdv": rng.integers(0, ndv, (nchan, nrow))}
maps = {k: torch.as_tensor(v.astype(np.int32), device=dev) for k, v in maps_h.items()}
v2i = torch.zeros(nchan, dtype=torch.int32, device=dev)
vis = torch.randn((nrow, nchan, npol), dtype=torch.complex128, device=dev)
wt = torch.ones((nrow, nchan, npol), dtype=torch.float64, device=dev)
cf = torch.randn((1, npol, nw, ndv, ndu, gv, gu), dtype=torch.complex128, device=dev)
grid = torch.zeros((1, npol, ny, nx), dtype=torch.complex128, device=dev)
sumwt = torch.zeros((1, npol), dtype=torch.float64, device=dev)


def timeit(m, v, w, reps=5):
    ts = []
    for _ in range(reps + 1):
        grid.zero_(); sumwt.zero_()
        torch.cuda.synchronize(); t0 = time.perf_counter()
        kernels.grid_cf(m, v2i, v, w, cf, grid, sumwt)
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    return np.median(ts[1:]) * 1e3


t = timeit(maps, vis, wt)
ref = grid.clone()
print(f"given order: {t:.2f} ms = {nrow / t / 1e3:.0f} Mvis/s", flush=True)
for T in (8, 16, 32, 64):
    key = (maps["pv"][0].long() // T) * (nx // T + 1) + maps["pu"][0].long() // T
    torch.cuda.synchronize(); t0 = time.perf_counter()
    order = torch.argsort(key)
    torch.cuda.synchronize(); ts = (time.perf_counter() - t0) * 1e3
    m2 = {k: v[:, order].contiguous() for k, v in maps.items()}
    t2 = timeit(m2, vis[order].contiguous(), wt[order].contiguous())
    err = float((grid - ref).abs().max() / ref.abs().max())
    print(f"tile {T}: sort {ts:.2f} ms, grid {t2:.2f} ms = {nrow / t2 / 1e3:.0f} Mvis/s, "
          f"max rel diff {err:.1e}", flush=True)
