"""C4 per-rank measurement on one GPU (BASELINE.json configs[3]).

SKA-LOW 512 stations, 400 times over 8 h, 256 channels over 50-350 MHz sharded
by channel over 8 GPUs: this runs ONE rank's shard (32 interleaved channels =
1.67 Gvis) through the w-stacking invert onto the 8192^2 image (16384^2 grid)
and prints stage times, plane geometry and the per-GPU rate.  The 8-GPU job
adds one all-reduce of the 8192^2 fp64 image (parallel.invert_sharded).

usage: python scripts/bench_c4_shard.py [--ntimes 400] [--nchan 32] [--npix 8192]
"""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
import numpy as np, torch
from ska_sdp_func_python_amd import kernels, parallel, simulation

ap = argparse.ArgumentParser()
ap.add_argument("--ntimes", type=int, default=400)
ap.add_argument("--nchan", type=int, default=32, help="channels of this shard")
ap.add_argument("--nchan-total", type=int, default=256)
ap.add_argument("--npix", type=int, default=8192)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--layout", choices=("interleaved", "block"), default="interleaved",
                help="channel sharding: every 8th channel, or a contiguous 1/8 of the band")
ap.add_argument("--rank", type=int, default=0, help="which shard (block layout: 7 = top band)")
ap.add_argument("--predict", action="store_true", help="also time dirty2ms (predict) of the image")
a = ap.parse_args()
dev = torch.device("cuda:0")
world = a.nchan_total // a.nchan
chans = (parallel.interleaved_channels(a.nchan_total, a.rank, world) if a.layout == "interleaved"
         else np.arange(a.rank * a.nchan, (a.rank + 1) * a.nchan))
t0 = time.perf_counter()
obs = simulation.device_observation(a.ntimes, a.nchan, 50e6, 350e6, config="LOW", device=dev,
                                    nchan_total=a.nchan_total, channels=chans)
torch.cuda.synchronize()
print(f"generated {obs['nrow']} rows x {len(chans)} chans in {time.perf_counter() - t0:.1f} s", flush=True)
cell = 0.25 / obs["umax"]
nvis = obs["nrow"] * len(chans)
kernels.set_stage_timing(True)
res = []
for it in range(a.reps + 1):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    img, info = kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], a.npix, a.npix,
                                 cell, cell, 1e-12, True, flip_uw=True)
    torch.cuda.synchronize(); dt = time.perf_counter() - t0
    print(f"rep {it}: {dt * 1e3:.1f} ms {info}", flush=True)
    if it > 0:
        res.append((dt, info))
dt = float(np.mean([r[0] for r in res]))
info = res[-1][1]
print(json.dumps({"config": "C4 shard: SKA-LOW 512 st, %d chan of %d (%s, rank %d), %d times, %d^2 image"
                  % (len(chans), a.nchan_total, a.layout, a.rank, a.ntimes, a.npix),
                  "nvis": nvis, "ms": round(dt * 1e3, 2), "Mvis_s_per_gpu": round(nvis / dt / 1e6, 1),
                  "stages_ms": {k: round(info[k], 2) for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")},
                  "nplanes": info["nplanes"], "plane_chunk": info["plane_chunk"],
                  "ngrid": info["ngrid_x"], "bucket": info["bucket"], "nitems": info["nitems"],
                  "support": info["support"], "grid_launches": info["grid_launches"],
                  "gpu_mem_peak_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1)}), flush=True)
if a.predict:
    pres = []
    for it in range(a.reps + 1):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        v, pinfo = kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell, 1e-12, True,
                                    flip_uw=True)
        torch.cuda.synchronize(); pdt = time.perf_counter() - t0
        if it > 0:
            pres.append(pdt)
        del v
    pdt = float(np.mean(pres))
    print(json.dumps({"predict_ms": round(pdt * 1e3, 2), "predict_Mvis_s_per_gpu": round(nvis / pdt / 1e6, 1),
                      "stages_ms": {k: round(pinfo[k], 2) for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")}}),
          flush=True)
