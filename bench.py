#!/usr/bin/env python
"""Headline benchmark: w-stacking invert (ms2dirty) throughput on MI355X.

metric  "Mvis/s gridded (invert, 8k^2 w-stack grid) at 1/2/4/8 MI355X"
        (BASELINE.json), measured on configs[1] (C2): SKA-MID-like 197 dishes,
        64 channels x 100 times = 123.6 Mvis per GPU, 4096^2 image on the
        8192^2 (sigma = 2) w-stacked grid, cell = 0.25 / u_max, epsilon 1e-7:
        the fp32 NUFFT at support W = 8 (north_star's stated fp32 tolerance,
        relative RMS < 1e-5; measured 9e-7 against the fp64 reference).  The
        reference's default 1e-12 runs the fp64 NUFFT.
step    one invert of the rank's visibilities, resident in HBM: bucketing,
        w-stack gridding, per-plane FFT, w-screen / grid-correction, the RCCL
        all-reduce of the dirty image and sumwt, and the sumwt normalisation
        (imaging/ng.py:146-294 + imaging/base.py:95-155).
scaling weak: every rank grids its own 64 channels; the N-GPU job is the same
        array observed in 64*N channels interleaved over 0.95-1.76 GHz, so
        every shard has the same uv extent and w-plane count.

Rank 0 prints ONE JSON line.  With --gpus 1 (the default) and the default
config it also carries one object per other configuration, each with its own
steps, timing, `roofline` and `cpu_baseline` (--no-extra skips them):
  "c4_n1"  configs[3] at N = 1: the whole 256-channel SKA-LOW band (13.4 Gvis,
           8192^2 image, 16384^2 grid, 71 w planes) streamed through
           sdp_hip_ms2dirty_batch -- the metric's own 8k^2 configuration;
  "c3"     configs[2]: the 1000-component x 10 Mvis sky-component DFT;
  "c5"     configs[4]: the 256,000-solve StefCal batch.
`roofline` uses the dominant kernel (k_grid):
its launch duration is measured live with HIP events recorded by the C ABI
on the stream the kernel runs on (sdp_hip_set_stage_timing); its algorithmic
bytes are N_vis * 12.375 B (c64 vis + f32 weight + f64 uvw per row / nchan,
SURVEY.md §8(d)) + n_planes * 8192^2 * 8 B (one write of the c64 grid).
`cpu_baseline` times oracle/wgrid_cpu.c (C + OpenMP restatement of the same
algorithm; ducc0 itself is unavailable) on a bounded sample -- rank 0, N=1.
"""

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "Mvis/s gridded (invert, 8k^2 w-stack grid) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3       # fp32 vector (packed FMA) peak
NCHAN_PER_GPU, NTIMES, NPIX = 64, 100, 4096
F_LO, F_HI = 0.95e9, 1.76e9
EPS_REQUESTED = 1e-7  # the fp32 NUFFT, W = 8 (epsilon < 1e-7 selects fp64)
EPS_REFERENCE = 1e-12  # invert_ng's default (ng.py:178): the fp64 NUFFT, W = 13
FP64_PEAK_TFLOPS = 78.6       # fp64 vector = fp64 matrix peak on gfx950


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nchan", type=int, default=NCHAN_PER_GPU, help="channels per GPU")
    ap.add_argument("--ntimes", type=int, default=NTIMES)
    ap.add_argument("--npix", type=int, default=NPIX)
    ap.add_argument("--cpu-chans", type=int, default=8,
                    help="channels in the cpu_baseline sample (0 = skip)")
    ap.add_argument("--no-api", action="store_true",
                    help="skip the invert_ng API (device / host Visibility) timings")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_k_grid.json"))
    ap.add_argument("--config", choices=("c2", "c3", "c4", "c5"), default="c2",
                    help="c2: configs[1], weak scaling (default); c3: configs[2], the sky-"
                         "component DFT; c4: configs[3], the SKA-LOW 256-channel band on the "
                         "8192^2 image, strong scaling; c5: configs[4], the StefCal batch")
    ap.add_argument("--c5-times", type=int, default=1000,
                    help="c5: time samples of the 512-station x 256-channel solve (1000 = C5)")
    ap.add_argument("--c4-batch", type=int, default=40,
                    help="c4: max channels per streamed batch of a rank's block (a block is "
                         "split into that many near-equal batches; 40 keeps one batch per "
                         "rank at N = 8 where the visibility cap below allows)")
    ap.add_argument("--c4-batch-gvis", type=float, default=1.8,
                    help="c4: max Gvis per batch -- the 4-padded record copy of the "
                         "large-grid invert (~38 B per visibility with the 16-B records "
                         "and ranks) must fit beside the 71 resident 16384^2 planes")
    ap.add_argument("--cu-split", default=os.environ.get("SDP_BENCH_CU_SPLIT", "alt"),
                    help="c2 pipelined: the two streams on disjoint CU masks ('alt', default: "
                         "alternate CUs, hipExtStreamCreateWithCUMask; 'half': the low / high "
                         "halves; '' = both streams on every CU).  C2: alt 11,717 vs 11,461 "
                         "Mvis/s unmasked, half 11,213 (profiles/r05_cu_split.txt)")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="c2: run the steps back to back on one stream (default: two streams "
                         "and two library scratch slots, consecutive inverts overlapping)")
    ap.add_argument("--no-extra", action="store_true",
                    help="default config at N=1: skip the c4_n1 / c3 / c5 objects")
    ap.add_argument("--extra-steps", type=int, default=2,
                    help="timed steps of the c4_n1 and c5 objects (c3 uses --steps)")
    ap.add_argument("--c4-cpu-chans", type=int, default=2,
                    help="c4: channels in the cpu_baseline sample (0 = skip)")
    ap.add_argument("--c4-traffic", default=os.path.join(ROOT, "profiles", "traffic_c4_k_grid.json"))
    ap.add_argument("--partition", choices=("auto", "wrow", "chan", "wslab"), default="auto",
                    help="c4 with N > 1: 'auto' (default) -- 'chan' at N = 2, 'wrow' at N >= 4 "
                         "(the faster of the two per world size on the one-GPU emulation: "
                         "2-way chan 1.89x vs wrow 1.78x, 4-way wrow 3.71x vs chan 3.35x, "
                         "8-way wrow 7.53x vs chan 5.36x; profiles/r03_c4_chan_24way.jsonl, "
                         "r03_c4_wrow_scaling_final_summary.txt); 'wrow' -- ranks own contiguous w intervals "
                         "of the rows and grid all channels of their rows, each with its own "
                         "w planes (parallel.wrow_partition); 'chan' -- cost-balanced contiguous "
                         "channel blocks (parallel.balanced_channel_blocks; the top block holds "
                         "every plane); 'wslab' -- every rank scans the band and grids its slab "
                         "of the band's w planes (parallel.wslab_partition; 2.6x at N = 8: the "
                         "w ~ 0 plane holds 38 %% of the visibilities) -- DESIGN.md §6")
    ap.add_argument("--c4-api", action="store_true",
                    help="C4 through the drop-in API: each rank builds a Visibility of its own "
                         "block (resident c64 vis, unit weights) and calls invert_ng(..., "
                         "shard='local'), which batches the block's channels and all-reduces "
                         "the image and weights; needs --gpus >= 2 or --emulate")
    ap.add_argument("--emulate", default=None, metavar="RANK/WORLD",
                    help="c4 on one GPU: run only rank RANK's block of a WORLD-way partition "
                         "(no collective), to measure per-rank times")
    return ap.parse_args()


def cpu_baseline(args, umax, nchan_total):
    """oracle/wgrid_cpu.c on bounded C2 samples: the sample's gridding time is
    scaled to the full visibility count and its per-plane FFT + w-screen time
    counted once (the full job has the same planes), giving the CPU's full-C2
    invert rate.  `value`: matched precision (fp32 taps and planes, W = 8,
    what the GPU computes) on all host cores the process may use (<= 16).
    `variants`: the same at the reference's default 4 threads (ng.py:58), and
    the reference's precision (epsilon 1e-12 -> W = 13, fp64 taps and planes,
    double_precision_accumulation=True, ng.py:240-256) at both thread counts."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wgrid_cpu
    from ska_sdp_func_python_amd import simulation
    fn, n_def, lat, dec = simulation.CONFIGS["MID"]
    en = fn(n_def, seed=1)
    ha = np.linspace(-0.5, 0.5, args.ntimes) * 8.0 * math.pi / 12.0
    uvw, _ = simulation.observe(en, math.radians(lat), math.radians(dec), ha)
    uvw = uvw.reshape(-1, 3) * np.array([-1.0, 1.0, -1.0])
    allf = np.linspace(F_LO, F_HI, nchan_total)
    cell = 0.25 / umax
    allcores = min(16, len(os.sched_getaffinity(0)))
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env > 0:
        allcores = min(allcores, env)
    nvis_full = uvw.shape[0] * args.nchan

    def run(nch, threads, precision):
        chans = np.linspace(0, nchan_total - 1, nch).round().astype(int)
        freq = allf[chans]
        rng = np.random.default_rng(2)
        ms = (rng.normal(size=(uvw.shape[0], nch))
              + 1j * rng.normal(size=(uvw.shape[0], nch))).astype(np.complex64)
        wgt = np.ones(ms.shape, np.float32)
        info = {}
        t0 = time.perf_counter()
        # matched precision: W = 8 fp32; the reference's: epsilon 1e-12 (W = 13, fp64)
        eps = EPS_REQUESTED if precision == "single" else 1e-12
        _, tg, tf = wgrid_cpu.ms2dirty(uvw, freq, ms, wgt, args.npix, args.npix, cell, cell,
                                       eps, True, nthreads=threads, precision=precision,
                                       info=info)
        wall = time.perf_counter() - t0
        t_full = (wall - tf) * nvis_full / ms.size + tf
        return {"value": round(nvis_full / t_full / 1e6, 4), "cores": threads,
                "precision": precision, "support": info["support"], "nplanes": info["nplanes"],
                "sample": f"{nch} of {args.nchan} channels ({ms.size / 1e6:.2f} Mvis): {wall:.1f} s "
                          f"wall, {tf:.1f} s FFT+screen"}

    main = run(args.cpu_chans, allcores, "single")
    variants = [run(max(1, args.cpu_chans // 2), 4, "single"),
                run(max(1, args.cpu_chans // 2), allcores, "double"),
                run(max(1, args.cpu_chans // 4), 4, "double")]
    return {"value": main["value"], "unit": "Mvis/s", "cores": allcores, "kind": "port",
            "sample": ("oracle/wgrid_cpu.c (C+OpenMP w-stacking restatement, load-balanced "
                       "tile tasks; ducc0 absent), matched precision (fp32, W=8) on "
                       + main["sample"] + "; full-job rate = gridding scaled to all "
                       f"{nvis_full / 1e6:.1f} Mvis + FFT/screen once"),
            "variants": variants}


def api_rates(args, obs, cell):
    """invert_ng through the reference-shaped API (datamodels-shim Visibility
    with the datamodels' dtypes: vis c128, weights f64, flags int64) on the
    bench workload: device-resident arrays, and host numpy arrays copied to
    the device inside the call (PCIe-inclusive; never the headline value)."""
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.imaging import invert_ng, predict_ng
    dev = obs["uvw"].device
    nrow, nchan = obs["nrow"], obs["vis"].shape[1]
    nb = 197 * 196 // 2
    nt = nrow // nb
    shape = (nt, nb, nchan, 1)
    pc = dm.SkyCoord(0.0, math.radians(-45.0))
    freq = obs["freq"].cpu().numpy()

    def make(arrs):
        return dm.Visibility.constructor(
            frequency=freq, channel_bandwidth=np.full(nchan, 1e6), phasecentre=pc,
            uvw=arrs["uvw"], time=np.arange(nt, dtype=float), vis=arrs["vis"],
            weight=arrs["w"], imaging_weight=arrs["w"], flags=arrs["f"],
            baselines=np.stack(np.triu_indices(197, 1), 1), polarisation_frame=dm.PolarisationFrame("stokesI"))

    d = {"uvw": obs["uvw"].reshape(nt, nb, 3),
         "vis": obs["vis"].to(torch.complex128).reshape(shape),
         "w": torch.ones(shape, dtype=torch.float64, device=dev),
         "f": torch.zeros(shape, dtype=torch.int64, device=dev)}
    model = dm.create_image(args.npix, cell, pc, frequency=float(freq.mean()),
                            channel_bandwidth=float(2 * (freq.max() - freq.min()) + 1e6), nchan=1)

    def timed(bvis, reps=2):
        invert_ng(bvis, model, epsilon=EPS_REQUESTED)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            invert_ng(bvis, model, epsilon=EPS_REQUESTED)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        return min(ts)

    t_dev = timed(make(d))
    nvis = nrow * nchan
    out = {"invert_ng_device_visibility_ms": round(t_dev * 1e3, 2)}

    def both(bvis, mdl):
        """(default, serial) ms of one invert_ng: invert_ng's own choice (an
        MFS image's pols share one bucketing; a cube's channels alternate
        two streams and scratch slots), and SDP_HIP_OVERLAP=0 (every call
        on one stream, pols still sharing)."""
        r = {}
        for tag, val in (("default", "1"), ("serial", "0")):
            os.environ["SDP_HIP_OVERLAP"] = val
            invert_ng(bvis, mdl, epsilon=EPS_REQUESTED)
            ts = []
            for _ in range(2):
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                invert_ng(bvis, mdl, epsilon=EPS_REQUESTED)
                torch.cuda.synchronize(dev)
                ts.append(time.perf_counter() - t0)
            r[tag] = min(ts)
        os.environ.pop("SDP_HIP_OVERLAP", None)
        return r

    # a 4-pol MFS image (linear vis -> stokesIQUV: 4 pols of 123.6 Mvis in one library call)
    s4 = (nt, nb, nchan, 4)
    v4 = obs["vis"].to(torch.complex128).reshape(nt, nb, nchan, 1).expand(s4).contiguous()
    d4 = {"uvw": d["uvw"], "vis": v4, "w": torch.ones(s4, dtype=torch.float64, device=dev),
          "f": torch.zeros(s4, dtype=torch.int64, device=dev)}
    b4 = dm.Visibility.constructor(
        frequency=freq, channel_bandwidth=np.full(nchan, 1e6), phasecentre=pc, uvw=d4["uvw"],
        time=np.arange(nt, dtype=float), vis=d4["vis"], weight=d4["w"], imaging_weight=d4["w"],
        flags=d4["f"], baselines=np.stack(np.triu_indices(197, 1), 1),
        polarisation_frame=dm.PolarisationFrame("linear"))
    m4 = dm.create_image(args.npix, cell, pc, polarisation_frame=dm.PolarisationFrame("stokesIQUV"),
                         frequency=float(freq.mean()),
                         channel_bandwidth=float(2 * (freq.max() - freq.min()) + 1e6), nchan=1)
    r4 = both(b4, m4)
    # predict_ng of a 4-pol model into that Visibility (one call for every pol)
    m4p = m4.copy(deep=True)
    m4p["pixels"].data = torch.randn(tuple(m4["pixels"].data.shape), dtype=torch.float64,
                                     device=dev)
    predict_ng(b4, m4p, epsilon=EPS_REQUESTED)
    ts = []
    for _ in range(2):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        predict_ng(b4, m4p, epsilon=EPS_REQUESTED)
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    tp4 = min(ts)
    del m4p
    # the same at the reference's default epsilon (fp64 NUFFT; each pol its
    # own two-level bucketing and MFMA gridder, pipelined)
    invert_ng(b4, m4, epsilon=EPS_REFERENCE)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    invert_ng(b4, m4, epsilon=EPS_REFERENCE)
    torch.cuda.synchronize(dev)
    t4_64 = time.perf_counter() - t0
    del b4, d4, v4
    torch.cuda.empty_cache()
    # a 16-channel cube (stokesI; 4 visibility channels per image channel, one
    # NUFFT call per image channel)
    dfc = float(freq[1] - freq[0])
    mc = dm.create_image(args.npix, cell, pc, frequency=float(freq[:4].mean()),
                         channel_bandwidth=4 * dfc, nchan=16)
    rc = both(make(d), mc)
    out.update({
        "invert_ng_4pol_ms": round(r4["default"] * 1e3, 2),
        "invert_ng_4pol_serial_ms": round(r4["serial"] * 1e3, 2),
        "invert_ng_4pol_Mvis_s": round(4 * nvis / r4["default"] / 1e6, 1),
        "invert_ng_4pol_eps1e-12_ms": round(t4_64 * 1e3, 2),
        "predict_ng_4pol_ms": round(tp4 * 1e3, 2),
        "invert_ng_cube16_ms": round(rc["default"] * 1e3, 2),
        "invert_ng_cube16_serial_ms": round(rc["serial"] * 1e3, 2),
        "invert_ng_cube16_Mvis_s": round(nvis / rc["default"] / 1e6, 1)})
    h = {k: v.cpu().numpy() for k, v in d.items()}
    del d
    torch.cuda.empty_cache()
    t_host = timed(make(h))
    out.update({"invert_ng_host_visibility_ms": round(t_host * 1e3, 2),
                "host_visibility_Mvis_s": round(nvis / t_host / 1e6, 1),
                "note": "reference-shaped invert_ng on a c128/f64/int64 Visibility; the host "
                        "figure includes the H2D copies of ~5 GB (PCIe-inclusive) and the image "
                        "D2H; 4pol: a linear-frame Visibility imaged to stokesIQUV (one library "
                        "call: one bucketing and value pass for the 4 pols; predict_ng_4pol: a random stokesIQUV model into "
                        "it, one library call for every pol); cube16: 64 vis channels onto a 16-channel "
                        "image (one call per image channel's run of 4 vis channels, 16 calls "
                        "pipelined over two streams); 'serial' = "
                        "SDP_HIP_OVERLAP=0 (one stream)"})
    return out


def _timed_calls(fn, steps, warmup, dev):
    """Wall time of `steps` calls of fn (after `warmup`), one stream, then one
    more call with the C ABI's stage timing on (HIP events around every
    stage on the launch stream) for its stage times."""
    from ska_sdp_func_python_amd import kernels
    kernels.set_stage_timing(False)
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / steps
    kernels.set_stage_timing(True)
    infos = [fn()[1] for _ in range(2)]
    kernels.set_stage_timing(False)
    return el, infos[-1]


def _traffic(name):
    """PMC bytes per launch of a kernel from profiles/<name> (scripts/
    pmc_traffic.sh), or None when no such measurement is committed."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("bytes_per_launch")


def c2_predict_and_fp64(args, obs, cell, dev, cpu):
    """Two more C2 objects (SURVEY.md §8 a2 and the reference's default
    precision), each with its own roofline and CPU baseline:

    * c2_predict -- dirty2ms (predict_ng's NUFFT, ng.py:95-129) of a random
      4096^2 model onto the 123.6 Mvis at epsilon 1e-7 (fp32, W = 8);
      roofline of the degridder k_degrid_mfma: the same algorithmic bytes as
      the gridder (12.375 B per visibility + the planes read once);
      cpu_baseline = oracle/wgrid_cpu.c dirty2ms (fp32, W = 8).
    * c2_fp64 -- ms2dirty at the reference's default epsilon 1e-12 (ng.py:178,
      double_precision_accumulation=True): the fp64 NUFFT (W = 13, c128
      planes, fp64 taps); roofline of k_grid_f64 against HBM and against the
      fp64 peak (4 W^3 flops per visibility); cpu_baseline = the fp64
      variant of the C2 CPU baseline (same restatement at W = 13)."""
    from ska_sdp_func_python_amd import kernels
    nvis = obs["nrow"] * obs["freq"].shape[0]
    nchan = obs["freq"].shape[0]
    g = torch.Generator(device=dev)
    g.manual_seed(77)
    img = torch.randn((args.npix, args.npix), generator=g, device=dev, dtype=torch.float64)
    vout = torch.empty((obs["nrow"], nchan), dtype=torch.complex64, device=dev)

    def pred():
        return kernels.dirty2ms(obs["uvw"], obs["freq"], img, None, cell, cell, EPS_REQUESTED,
                                True, flip_uw=True, out=vout)
    el, info = _timed_calls(pred, args.steps, 2, dev)
    alg = nvis * (8 + 4 + 24.0 / nchan) + info["nplanes"] * info["ngrid_x"] * info["ngrid_y"] * 8
    kms = info["ms_grid"] / max(1, info["grid_launches"])
    ach = alg / max(1, info["grid_launches"]) / (kms * 1e-3) / 1e9
    pcpu = None
    if args.cpu_chans > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import wgrid_cpu
        nch = max(1, args.cpu_chans // 2)
        idx = np.linspace(0, nchan - 1, nch).round().astype(int)
        uvw_h = obs["uvw"].cpu().numpy() * np.array([-1.0, 1.0, -1.0])
        f_h = obs["freq"].cpu().numpy()[idx]
        threads = cpu["cores"] if cpu else min(16, len(os.sched_getaffinity(0)))
        t0 = time.perf_counter()
        _, tg, tf = wgrid_cpu.dirty2ms(uvw_h, f_h, img.cpu().numpy(), None, cell, cell,
                                       EPS_REQUESTED, True, nthreads=threads, precision="single")
        wall = time.perf_counter() - t0
        t_full = (wall - tf) * nvis / (uvw_h.shape[0] * nch) + tf
        pcpu = {"value": round(nvis / t_full / 1e6, 4), "unit": "Mvis/s", "cores": threads,
                "kind": "port",
                "sample": f"oracle/wgrid_cpu.c dirty2ms (fp32, W=8) on {nch} of {nchan} channels "
                          f"({uvw_h.shape[0] * nch / 1e6:.2f} Mvis): {wall:.1f} s wall, {tf:.1f} s "
                          "FFT+screen; degridding scaled to all visibilities + FFT/screen once"}
    predict = {
        "metric": "Mvis/s degridded (predict, 8k^2 w-stack grid)", "value": round(nvis / el / 1e6, 3),
        "unit": "Mvis/s", "n_gpus": 1, "steps": args.steps, "ms_per_step": round(el * 1e3, 3),
        "higher_is_better": True, "dtype": "f32",
        "config": {"workload": "C2 predict: dirty2ms of a 4096^2 model onto 123.6 Mvis, 8192^2 "
                               "w-stack grid, epsilon 1e-7 (W = 8)", "nplanes": info["nplanes"]},
        "stages_ms": {k: round(float(info[k]), 3) for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")},
        "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4),
                     "traffic": _traffic("traffic_k_degrid.json"),
                     "kernel": f"k_degrid_mfma<{info['support']},true>", "kernel_ms": round(kms, 4),
                     "alg_bytes_per_launch": int(alg / max(1, info["grid_launches"]))},
        "cpu_baseline": pcpu}
    del vout
    out = torch.empty((args.npix, args.npix), dtype=torch.float64, device=dev)

    def inv64():
        return kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], args.npix, args.npix,
                                cell, cell, EPS_REFERENCE, True, flip_uw=True, out=out)
    el, info = _timed_calls(inv64, max(2, args.extra_steps), 1, dev)
    W = info["support"]
    alg = nvis * (8 + 4 + 24.0 / nchan) + info["nplanes"] * info["ngrid_x"] * info["ngrid_y"] * 16
    kms = info["ms_grid"] / max(1, info["grid_launches"])
    ach = alg / max(1, info["grid_launches"]) / (kms * 1e-3) / 1e9
    tfl = nvis * 4 * W ** 3 / (info["ms_grid"] * 1e-3) / 1e12
    c64 = None
    if cpu and len(cpu.get("variants", [])) > 1:
        v = cpu["variants"][1]
        c64 = {"value": v["value"], "unit": "Mvis/s", "cores": v["cores"], "kind": "port",
               "sample": "oracle/wgrid_cpu.c at the reference's precision (fp64, W = "
                         f"{v['support']}, {v['nplanes']} planes), {v['sample']}"}
    fp64 = {
        "metric": METRIC + " at the reference's default epsilon 1e-12 (fp64 NUFFT)",
        "value": round(nvis / el / 1e6, 3), "unit": "Mvis/s", "n_gpus": 1,
        "steps": max(2, args.extra_steps), "ms_per_step": round(el * 1e3, 3),
        "higher_is_better": True, "dtype": "f64",
        "config": {"workload": "C2 invert at epsilon 1e-12: 123.6 Mvis, 4096^2 image, 8192^2 "
                               "w-stack grid", "support": W, "nplanes": info["nplanes"],
                   "epsilon_requested": EPS_REFERENCE, "fp64": info["fp64"]},
        "stages_ms": {k: round(float(info[k]), 3) for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")},
        "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4),
                     "traffic": _traffic("traffic_k_grid_f64.json"),
                     "kernel": f"k_grid_f64_mfma<{W},true>", "kernel_ms": round(kms, 4),
                     "alg_bytes_per_launch": int(alg / max(1, info["grid_launches"])),
                     "compute": {"achieved": round(tfl, 2), "peak": FP64_PEAK_TFLOPS,
                                 "unit": "TFLOP/s", "frac": round(tfl / FP64_PEAK_TFLOPS, 4),
                                 "note": "4 W^3 fp64 flops per visibility"}},
        "cpu_baseline": c64}
    del out
    # the fp64 predict (dirty2ms at 1e-12: k_degrid_f64_mfma), same model
    vout = torch.empty((obs["nrow"], nchan), dtype=torch.complex128, device=dev)

    def pred64():
        return kernels.dirty2ms(obs["uvw"], obs["freq"], img, None, cell, cell, EPS_REFERENCE,
                                True, flip_uw=True, out=vout)
    el, info = _timed_calls(pred64, max(2, args.extra_steps), 1, dev)
    kms = info["ms_grid"] / max(1, info["grid_launches"])
    fp64["predict"] = {
        "value": round(nvis / el / 1e6, 3), "unit": "Mvis/s", "ms_per_step": round(el * 1e3, 3),
        "stages_ms": {k: round(float(info[k]), 3) for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")},
        "kernel": f"k_degrid_f64_mfma<{info['support']},true>", "kernel_ms": round(kms, 4),
        "compute_TFLOP_s": round(nvis * 4 * info["support"] ** 3 / (info["ms_grid"] * 1e-3) / 1e12, 2)}
    del vout
    return {"c2_predict": predict, "c2_fp64": fp64}


# ---------------------------------------------------------------------------
# C4: SKA-LOW 512 stations x 400 times x 256 channels (13.4 Gvis), 8192^2 image
# ---------------------------------------------------------------------------
C4_NCHAN, C4_NTIMES, C4_NPIX, C4_FLO, C4_FHI = 256, 400, 8192, 50e6, 350e6


def c4_cpu_baseline(uvw_h, freqs, cell, nvis_total, nplanes_full, nchan_sample):
    """oracle/wgrid_cpu.c (C + OpenMP restatement of the w-stacking invert,
    matched fp32 precision, W = 8) on the `nchan_sample` lowest channels of
    the band at the full 8192^2 image: its per-visibility gridding time is
    extrapolated to all 13.4 Gvis and its per-plane FFT + w-screen time to the
    band's plane count (the full job grids every visibility once and
    transforms each of its planes once)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wgrid_cpu
    threads = min(16, len(os.sched_getaffinity(0)))
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env > 0:
        threads = min(threads, env)
    freq = freqs[:nchan_sample]
    rng = np.random.default_rng(4)
    ms = (rng.normal(size=(uvw_h.shape[0], nchan_sample))
          + 1j * rng.normal(size=(uvw_h.shape[0], nchan_sample))).astype(np.complex64)
    info = {}
    t0 = time.perf_counter()
    _, tg, tf = wgrid_cpu.ms2dirty(uvw_h * np.array([-1.0, 1.0, -1.0]), freq, ms, None, C4_NPIX,
                                   C4_NPIX, cell, cell, EPS_REQUESTED, True, nthreads=threads,
                                   precision="single", info=info)
    wall = time.perf_counter() - t0
    t_vis = (wall - tf) / ms.size
    t_plane = tf / max(1, info["nplanes"])
    t_full = t_vis * nvis_total + t_plane * nplanes_full
    return {"value": round(nvis_total / t_full / 1e6, 4), "unit": "Mvis/s", "cores": threads,
            "kind": "port",
            "sample": (f"oracle/wgrid_cpu.c (C+OpenMP w-stacking restatement; ducc0 absent), fp32 "
                       f"W={info['support']}, {nchan_sample} lowest channels x {uvw_h.shape[0]} rows "
                       f"({ms.size / 1e6:.1f} Mvis) on the 8192^2 image: {wall:.1f} s wall, "
                       f"{tf:.1f} s FFT+screen for {info['nplanes']} planes; extrapolated "
                       f"(gridding per visibility x {nvis_total / 1e9:.2f} Gvis + FFT/screen per "
                       f"plane x {nplanes_full} planes) = {t_full:.0f} s for the band")}


def run_c4(args, world, rank, local, dev, emulated=False, sub=False):
    """Strong scaling of configs[3]: the fixed 256-channel band is split into
    `world` contiguous channel blocks balanced by the measured cost model
    (parallel.balanced_channel_blocks); each rank streams its block through
    one set of resident w planes in batches of --c4-batch channels
    (kernels.ms2dirty_batch: one plane layout, one FFT pass per rank), then
    one all-reduce of the 8192^2 fp64 image.  At N = 1 the single GPU
    streams all 256 channels through the band's 71 planes.  Inputs: the
    rank's uvw (52.3 M rows) resident; the batches' visibilities are resident
    when they fit (N >= 4) and the step is timed as one bracket, else each
    batch is generated on device between timed segments (the sum of the
    segments, then the max over ranks, is the step time).

    `roofline` (dominant kernel: the gridder, summed over the batch launches):
    algorithmic bytes = every visibility once (8 B c64, unit weights) + the
    rows' uvw once per batch (24 B) + ONE write of the band's planes
    (nplanes x 16384^2 x 8 B) per invert -- the planes stay resident across
    the batches, so they are charged once, not once per batch; `compute` the
    same launches against the fp32 MFMA peak (4 W^3 flops per visibility).
    `sub` returns the line as a dict (the default bench's "c4_n1" object)."""
    from ska_sdp_func_python_amd import kernels, parallel, simulation
    freqs = np.linspace(C4_FLO, C4_FHI, C4_NCHAN)
    if args.partition == "auto":
        args.partition = "chan" if world <= 2 else "wrow"
    wslab = args.partition == "wslab" and world > 1  # (N = 1: the whole band, no slab)
    wrow = args.partition == "wrow" and world > 1
    blocks = ([(0, C4_NCHAN)] * world if wslab or wrow
              else parallel.balanced_channel_blocks(freqs, world))
    lo, hi = blocks[rank]
    obs = simulation.device_observation(C4_NTIMES, 1, C4_FLO, C4_FHI, config="LOW", seed=0,
                                        device=dev, nchan_total=C4_NCHAN, channels=[lo])
    uvw, nrow = obs["uvw"], obs["nrow"]
    row_costs = None
    if wrow:
        # the rank's rows: a contiguous interval of the rows' w (the imaging
        # sign, flip_uw), cut by the cost model over the band's plane spacing
        cell0 = 0.25 / obs["umax"]
        lay0 = kernels.wstack_layout(kernels.uvw_bounds(uvw, torch.as_tensor(freqs, device=dev)),
                                     C4_NPIX, C4_NPIX, cell0, cell0, EPS_REQUESTED, True,
                                     flip_uw=True)
        order, cuts, row_costs = parallel.wrow_partition((-uvw[:, 2]).cpu().numpy(), freqs, world,
                                                         lay0["dw"], lay0["support"])
        rows = torch.as_tensor(order[cuts[rank]:cuts[rank + 1]], device=dev)
        uvw = uvw[rows].contiguous()
        nrow = int(rows.numel())
        del rows
    nb = max(1, 0 if wrow else -(-(hi - lo) // args.c4_batch),
             math.ceil(nrow * (hi - lo) / (args.c4_batch_gvis * 1e9)))
    cuts = [lo + (hi - lo) * i // nb for i in range(nb + 1)]
    batches = list(zip(cuts[:-1], cuts[1:]))
    del obs["vis"], obs["wgt"]
    cell = 0.25 / obs["umax"]
    freq_all = torch.as_tensor(freqs, device=dev)
    local_freq = freq_all[lo:hi]
    bounds, slab, slabs, layout, hist = None, None, None, None, None
    if wslab:
        # the band's plane layout (identical on every rank) and this rank's slab
        bounds = kernels.merge_bounds(*[kernels.uvw_bounds(uvw, freq_all[a:e]) for a, e in batches])
        layout = kernels.wstack_layout(bounds, C4_NPIX, C4_NPIX, cell, cell, EPS_REQUESTED, True,
                                       flip_uw=True)
        hist = parallel.first_plane_histogram(uvw, freqs, layout)
        slabs = parallel.wslab_partition(hist, world, layout["support"])
        slab = slabs[rank]
    resident = world >= 4 and not wslab  # (wrow: ~14 GB of c64 per rank at N = 8)
    gen = torch.Generator(device=dev)
    steps = args.extra_steps if sub else args.steps
    warmup = min(args.warmup, 1) if sub else args.warmup

    def make_vis(a, e):
        gen.manual_seed(7919 * (0 if wslab else rank) + a)  # (w slabs: one band, every rank)
        return torch.randn((nrow, e - a), generator=gen, device=dev, dtype=torch.complex64)

    if args.c4_api:
        return run_c4_api(args, world, rank, local, dev, uvw, nrow, lo, hi, freqs, obs["umax"],
                          batches, make_vis, emulated, sub)
    store = {(a, e): make_vis(a, e) for a, e in batches} if resident else {}

    def vis_of_block(a, e):
        return store[(a + lo, e + lo)] if resident else make_vis(a + lo, e + lo)

    rel = [(a - lo, e - lo) for a, e in batches]
    out = torch.zeros((C4_NPIX, C4_NPIX), dtype=torch.float64, device=dev)
    nvis_rank = int(hist[slab[0]:slab[1]].sum()) if wslab else nrow * (hi - lo)
    seg = {"t": 0.0}

    class Seg:
        def __enter__(self):
            torch.cuda.synchronize(dev)
            self.t0 = time.perf_counter()

        def __exit__(self, *a):
            torch.cuda.synchronize(dev)
            seg["t"] += time.perf_counter() - self.t0
            return False

    dist_on = world > 1 and not emulated

    def barrier():
        if dist_on:
            dist.barrier(device_ids=[local])
        torch.cuda.synchronize(dev)

    infos = []

    def step(timer):
        out.zero_()
        parallel.invert_batched_shard(uvw, local_freq, vis_of_block, rel, C4_NPIX, cell, EPS_REQUESTED,
                                      True, flip_uw=True, out=out, timer=timer, bounds=bounds,
                                      slab=slab)

    def reduce():
        sw = torch.tensor([float(nrow * C4_NCHAN)], dtype=torch.float64, device=dev)
        if dist_on:
            dist.all_reduce(out, op=dist.ReduceOp.SUM)
        out.div_(sw)

    kernels.set_stage_timing(False)
    for _ in range(warmup):
        step(None)
        reduce()
    barrier()
    if resident:
        t0 = time.perf_counter()
        for _ in range(steps):
            step(None)
            reduce()
        barrier()
        elapsed = time.perf_counter() - t0
    else:
        for _ in range(steps):
            step(Seg)
            barrier()
            with Seg():
                reduce()
        barrier()
        elapsed = seg["t"]
    # one extra, untimed pass with stage timing for the kernel breakdown
    kernels.set_stage_timing(True)
    orig = kernels.ms2dirty_batch

    def spy(*a, **k):
        r = orig(*a, **k)
        infos.append(r[1])
        return r

    kernels.ms2dirty_batch = spy
    try:
        step(None)
    finally:
        kernels.ms2dirty_batch = orig
        kernels.set_stage_timing(False)
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = elapsed / steps * 1e3
    nvis_total = nrow * C4_NCHAN
    def model_ms(r):
        if wrow:
            return round(float(row_costs[r]), 1)
        if wslab:
            a, e = slabs[r]
            return round(parallel.wslab_cost(hist, a, e, layout["support"], float(hist.sum())), 1)
        return round(parallel.c4_block_cost(freqs[blocks[r][0]:blocks[r][1]]), 1)

    if emulated:
        print(json.dumps({"emulated_rank": rank, "world": world, "partition": args.partition,
                          "block": blocks[rank], "slab": slab,
                          "ms_per_step": round(ms_step, 3), "nvis_rank": nvis_rank,
                          "model_ms": model_ms(rank),
                          "stages_ms": {k: round(float(sum(i[k] for i in infos)), 3)
                                        for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")},
                          "note": "rank's block only; no all-reduce"}), flush=True)
        return None
    if rank != 0:
        return None
    value = nvis_total / (elapsed / steps) / 1e6
    info = infos[-1]
    W = info["support"]
    ms_grid = float(sum(i["ms_grid"] for i in infos))
    plane_bytes = info["nplanes"] * info["ngrid_x"] * info["ngrid_y"] * 8
    alg = nvis_rank * 8 + len(batches) * nrow * 24 + plane_bytes
    achieved = alg / (ms_grid * 1e-3) / 1e9 if ms_grid > 0 else None
    flops = nvis_rank * 4 * W ** 3
    traffic = None
    if os.path.exists(args.c4_traffic):
        with open(args.c4_traffic) as f:
            tr = json.load(f)
        # PMC bytes of all the batch launches of one invert (scripts/pmc_c4.sh),
        # the same span as `alg` and `kernel_ms_rank0`
        if tr.get("launches") == len(batches) and world == 1:
            traffic = tr.get("bytes_per_invert")
    model = [model_ms(r) for r in range(world)]
    cpu = None
    if world == 1 and args.c4_cpu_chans > 0:
        cpu = c4_cpu_baseline(uvw.cpu().numpy(), freqs, cell, nvis_total, info["nplanes"],
                              args.c4_cpu_chans)
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "Mvis/s", "n_gpus": world,
        "steps": steps, "warmup": warmup, "ms_per_step": round(ms_step, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (seeded SKA-LOW-like layout, N(0,1) c64 vis, unit weights, "
                "generated on device)",
        "config": {"workload": "C4: SKA-LOW 512 stations x 400 times x 256 chan (50-350 MHz) "
                               "= 13.4 Gvis, 8192^2 image, 16384^2 w-stack grid",
                   "nvis_total": nvis_total, "npix": C4_NPIX, "cell_rad": cell,
                   "partition": args.partition if world > 1 else "none",
                   "rank0_rows": nrow,
                   "channel_blocks": blocks if not wslab else None, "w_slabs": slabs,
                   "model_ms_per_rank": model,
                   "rank0_batches": len(batches), "inputs_resident": resident,
                   "support": W, "nplanes_rank0": info["nplanes"],
                   "parallelism": (f"w slabs x{world} (each rank scans the band, grids its "
                                   "slab's first planes), streamed batches, 1 all-reduce"
                                   if wslab else
                                   f"row w-intervals x{world} (all channels of the rank's rows, "
                                   "own w planes), streamed batches, 1 all-reduce" if wrow else
                                   f"channel blocks x{world}, streamed batches, 1 all-reduce")},
        "stages_ms_rank0": {k: round(float(sum(i[k] for i in infos)), 3)
                            for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2) if achieved else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic,
                     "kernel": (f"k_grid_mfma_pad<{W},true> (sub-sorted, 4-padded cells)"
                                if info.get("padded") else
                                f"k_grid_mfma<{W},true> (sub-sorted cells)"),
                     "kernel_ms_rank0": round(ms_grid, 3), "launches": len(batches),
                     "alg_bytes": int(alg),
                     "note": "vis 8 B + uvw 24 B per row per batch + the band's planes written "
                             "once per invert, over the summed gridding launches; traffic = "
                             "PMC bytes of those launches (profiles/traffic_c4_k_grid.json)",
                     "compute": {"achieved": round(flops / (ms_grid * 1e-3) / 1e12, 2),
                                 "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                                 "frac": round(flops / (ms_grid * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                                               4)}},
        "cpu_baseline": cpu,
    }
    if sub:
        return line
    print(json.dumps(line), flush=True)
    return None


def run_c4_api(args, world, rank, local, dev, uvw, nrow, lo, hi, freqs, umax, batches, make_vis,
               emulated, sub):
    """C4 through the reference-shaped API: the rank's block (its rows by w,
    or its channel block) as a Visibility of [1, nrow, nchan, 1] (resident c64
    visibilities generated with run_c4's seeds; weights and flags are
    zero-stride views: unit weights, no flags) and one
    invert_ng(vis, model, shard="local", epsilon=1e-7) per step -- the call a
    pipeline holding one observation in N blocks makes.  invert_ng grids the
    block in channel batches (SDP_HIP_MAX_CALL_GVIS) through one set of
    resident planes, all-reduces the image and sumwt (ng.py:288-292) and
    normalises.  Step time: barrier + synchronize around each call, max over
    ranks; the line's value = the band's visibilities / that time."""
    from ska_sdp_func_python_amd import datamodels as dm
    from ska_sdp_func_python_amd.imaging import invert_ng
    if args.partition == "wslab":
        raise SystemExit("--c4-api: a w-slab rank scans the whole band (no Visibility block)")
    if world == 1 and not emulated:
        raise SystemExit("--c4-api: the 107 GB band does not fit beside its 152 GB of planes on "
                         "one GPU; use --gpus >= 2 or --emulate r/N")
    nch = hi - lo
    vis = torch.empty((1, nrow, nch, 1), dtype=torch.complex64, device=dev)
    for a, e in batches:
        vis[0, :, a - lo:e - lo, 0] = make_vis(a, e)
    ones = torch.ones((1, 1, 1, 1), dtype=torch.float32, device=dev).expand(1, nrow, nch, 1)
    noflag = torch.zeros((1, 1, 1, 1), dtype=torch.int8, device=dev).expand(1, nrow, nch, 1)
    pc = dm.SkyCoord(0.0, -0.5)
    f = freqs[lo:hi]
    bv = dm.Visibility.constructor(frequency=f, channel_bandwidth=np.full(nch, 1.17e6),
                                   phasecentre=pc, uvw=uvw.view(1, nrow, 3), time=np.zeros(1),
                                   vis=vis, weight=ones, imaging_weight=ones, flags=noflag,
                                   integration_time=np.ones(1))
    cell = 0.25 / umax
    model = dm.create_image(C4_NPIX, cell, pc, frequency=float(np.mean(freqs)),
                            channel_bandwidth=float(2 * (freqs.max() - freqs.min()) + 1e6))
    kw = {"shard": "local"} if world > 1 and not emulated else {}
    dist_on = world > 1 and not emulated
    steps = args.extra_steps if sub else args.steps
    warmup = min(args.warmup, 1) if sub else args.warmup

    def barrier():
        if dist_on:
            dist.barrier(device_ids=[local])
        torch.cuda.synchronize(dev)

    res = None
    for _ in range(warmup):
        res = invert_ng(bv, model, epsilon=EPS_REQUESTED, **kw)
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        res = invert_ng(bv, model, epsilon=EPS_REQUESTED, **kw)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = elapsed / steps * 1e3
    sumwt = float(np.sum(res[1]))
    if emulated:
        print(json.dumps({"emulated_rank": rank, "world": world, "partition": args.partition,
                          "api": "invert_ng",
                          "block": (lo, hi), "rows": nrow, "ms_per_step": round(ms_step, 3),
                          "nvis_rank": nrow * nch, "sumwt": sumwt,
                          "note": "rank's block only; no all-reduce"}), flush=True)
        return None
    if rank != 0:
        return None
    nvis_total = int(round(sumwt))  # unit weights: the band's visibility count
    line = {
        "metric": METRIC, "value": round(nvis_total / (elapsed / steps) / 1e6, 3), "unit": "Mvis/s",
        "n_gpus": world, "steps": steps, "warmup": warmup, "ms_per_step": round(ms_step, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (seeded SKA-LOW-like layout, N(0,1) c64 vis, unit weights, generated "
                "on device, resident)",
        "config": {"workload": "C4 through invert_ng(shard='local'): SKA-LOW 512 stations x 400 "
                               "times x 256 chan = 13.4 Gvis, 8192^2 image, 16384^2 w-stack grid",
                   "api": "invert_ng", "partition": args.partition, "nvis_total": nvis_total,
                   "parallelism": f"{args.partition} x{world}, each rank's own Visibility block, "
                                  "invert_ng channel batches, 1 all-reduce (image + sumwt)"}}
    if sub:
        return line
    print(json.dumps(line), flush=True)
    return None


# ---------------------------------------------------------------------------
# C3: dft_skycomponent_visibility, 1000 point components x 10 Mvis
# ---------------------------------------------------------------------------
C3_NCOMP, C3_NTIMES = 1000, 518   # 19,306 SKA-MID baselines x 518 times = 10.0 Mvis


# k_dft_mfma's binding pipe, from a PMC pass of the same C3 launch
# (scripts/pmc_sets.sh dft6 ... -- scripts/dft_once.py, summarised into
# profiles/r06_dft_pmc.json): the SIMDs' VALU-active fraction
# (SQ_ACTIVE_INST_VALU, quad-cycles, over SIMDs x GRBM_GUI_ACTIVE cycles), the
# MFMA-busy fraction (they never overlap: SQ_VALU_MFMA_COEXEC_CYCLES = 0) and
# the instruction mix per 64 component-visibilities.  The per-component work
# is two transcendentals (v_sin_f32, v_cos_f32) plus v_fract_f64, one
# conversion and two packed-f32 FMAs on the VALU; the phase product is a
# quarter of a v_mfma_f64_16x16x4_f64 per 64.  The transcendental bound is
# the sincos issue alone (8 cycles each per wave64, MI355X_MICROARCH.md
# "vector-instruction ISSUE cost").
DFT_TRANS_CYC = 2 * 8
MI355X_SIMDS, MI355X_GHZ = 256 * 4, 2.4
DFT_PMC = os.path.join(ROOT, "profiles", "r06_dft_pmc.json")


def _dft_issue_roofline(compvis, k_ms):
    """The DFT against its binding pipe: the VALU issue (measured active
    fraction from the committed PMC pass) and the transcendental rate."""
    rate = compvis / (k_ms * 1e-3)
    lanes = MI355X_SIMDS * MI355X_GHZ * 1e9 * 64
    trans_peak = lanes / DFT_TRANS_CYC  # component-visibilities / s if only sincos issued
    out = {"achieved": round(rate / 1e12, 3), "unit": "T comp*vis/s",
           "sincos_peak": round(trans_peak / 1e12, 3), "sincos_frac": round(rate / trans_peak, 4)}
    try:
        pmc = json.load(open(DFT_PMC))
        for k in ("valu_active_frac", "mfma_busy_frac", "simd_busy_frac", "insts_per_64_compvis"):
            out[k] = pmc[k]
        out["pmc_kernel_ms"] = pmc["kernel_ms"]
        out["source"] = os.path.relpath(DFT_PMC, ROOT)
    except (OSError, KeyError, ValueError):
        pass
    out["note"] = ("binding pipe: the SIMDs' issue (measured on the same launch: VALU active "
                   "plus MFMA busy, which never overlap on gfx950, = simd_busy_frac); sincos: "
                   "2 transcendentals x 8 issue cycles per 64 comp*vis per SIMD, "
                   f"{MI355X_SIMDS} SIMDs at {MI355X_GHZ} GHz")
    return out


def run_c3(args, world, rank, dev, sub=False):
    """configs[2]: the point-component DFT (reference imaging/dft.py:135-183,
    dft_cpu_looped) of 1000 components onto 10.0 Mvis (one channel, stokesI,
    c64 output).  Rows are split across ranks (strong scaling, no
    collective: parallel.dft_sharded's partitioning).  `roofline` is the
    VALU count N_vis N_comp (6 + 8 npol) flops against the
    fp32 vector peak -- sincos excluded, so the fraction understates the
    issue rate; `cpu_baseline` is ref_oracle.dft_cpu_looped (the reference's
    loop restated in numpy) on 100 components x 200k visibilities."""
    from ska_sdp_func_python_amd import kernels, simulation
    rng = np.random.default_rng(3)
    fn_, n_def, lat, dec = simulation.CONFIGS["MID"]
    ha = np.linspace(-0.5, 0.5, C3_NTIMES) * 8.0 * math.pi / 12.0
    uvw_h, _ = simulation.observe(fn_(n_def, seed=1), math.radians(lat), math.radians(dec), ha)
    uvw_h = uvw_h.reshape(-1, 3)
    nvis_total = uvw_h.shape[0]
    lo, hi = nvis_total * rank // world, nvis_total * (rank + 1) // world
    uvw = torch.as_tensor(uvw_h[lo:hi], device=dev)
    freq_h = np.array([1.4e9])
    freq = torch.as_tensor(freq_h, device=dev)
    lm = rng.uniform(-0.05, 0.05, (C3_NCOMP, 2))
    dc_h = np.concatenate([lm, (np.sqrt(1 - (lm ** 2).sum(1)) - 1)[:, None]], 1)
    fl_h = rng.uniform(0.1, 10, (C3_NCOMP, 1, 1)).astype(complex)
    dc, fl = torch.as_tensor(dc_h, device=dev), torch.as_tensor(fl_h, device=dev)
    out = torch.empty((hi - lo, 1, 1), dtype=torch.complex64, device=dev)

    def step():
        kernels.dft_point(dc, fl, uvw, freq=freq, out=out)

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[dev.index])
        torch.cuda.synchronize(dev)

    warmup = max(1, args.warmup) if sub else args.warmup
    for _ in range(warmup):
        step()
    barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    barrier()
    elapsed = time.perf_counter() - t0
    k_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = elapsed / args.steps * 1e3
    if rank != 0:
        return
    flops = (hi - lo) * C3_NCOMP * (6 + 8 * 1)
    cpu = None
    if world == 1:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import ref_oracle as ro
        ns, nc = 200_000, 100
        uvwl = uvw_h[:ns, None, :] * (freq_h / 299792458.0)[None, :, None]
        tc0 = time.perf_counter()
        ro.dft_cpu_looped(dc_h[:nc], uvwl, fl_h[:nc])
        tc = time.perf_counter() - tc0
        cpu_rate = ns * nc / tc
        cpu = {"value": round(cpu_rate / 1e9, 5), "unit": "G comp*vis/s", "cores": 1,
               "kind": "port",
               "sample": f"oracle/ref_oracle.dft_cpu_looped (the reference's loop, numpy), {nc} "
                         f"comps x {ns} vis in {tc:.1f} s; the full C3 extrapolates to "
                         f"{nvis_total * C3_NCOMP / cpu_rate:.0f} s"}
    line = {
        "metric": "G comp*vis/s (dft_skycomponent_visibility, 1000 components x 10 Mvis)",
        "value": round(nvis_total * C3_NCOMP / (elapsed / args.steps) / 1e9, 2),
        "unit": "G comp*vis/s", "n_gpus": world, "steps": args.steps, "warmup": warmup,
        "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32 (fp64 phase)",
        "data": "synthetic (seeded SKA-MID-like layout, 1000 components |l|,|m| < 0.05, "
                "fluxes U(0.1, 10))",
        "config": {"workload": "C3: 1000 point components x 10.0 Mvis (19,306 baselines x 518 "
                               "times x 1 channel, stokesI), c64 output",
                   "nvis": nvis_total, "ncomp": C3_NCOMP,
                   "parallelism": f"rows x{world}, no collective"},
        "roofline": {"bound": "valu", "achieved": round(flops / (k_ms * 1e-3) / 1e12, 2),
                     "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(flops / (k_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS, 4),
                     "traffic": None, "kernel": "k_dft_mfma", "kernel_ms": round(k_ms, 4),
                     "note": "N_vis N_comp (6 + 8 npol) flops (SURVEY.md 8(d)), sincos excluded; "
                             "the fp64 phase product runs on v_mfma_f64_16x16x4_f64, the "
                             "VALU keeps sincos and the flux multiply-add (DESIGN.md 2)",
                     "issue": _dft_issue_roofline(nvis_total * C3_NCOMP, k_ms)},
        "cpu_baseline": cpu,
    }
    if sub:
        return line
    print(json.dumps(line), flush=True)


# ---------------------------------------------------------------------------
# C5: solve_gaintable StefCal, 512 stations x 256 channels x 1000 times
# ---------------------------------------------------------------------------
C5_NANTS, C5_NCHAN, C5_BATCH = 512, 256, 16


def run_c5(args, world, rank, dev, sub=False):
    """configs[4]: 256,000 per-(time, channel) StefCal solves (B jones, the
    reference's solvers.py:217-300 scalar itsubs path, niter 200, tol 1e-6)
    of 512 stations.  The inputs of the whole job (33.5 G baseline samples,
    0.8 TB as c128 + f64) exceed HBM, so the rank's times are solved in
    batches of 16 gain rows (4096 sub-solves); each batch's x_b and weights
    are generated on device between timed segments and the step time is the
    sum of the solve segments (max over ranks).  Times are split across ranks
    (strong scaling, no collective).  `roofline`: 12 B per baseline per
    sub-solve iteration over the timed solves against HBM
    peak; `cpu_baseline`: ref_oracle.stefcal_row (numpy restatement) on 2
    single-channel sub-solves."""
    from ska_sdp_func_python_amd import kernels
    ntime = args.c5_times
    t_lo, t_hi = ntime * rank // world, ntime * (rank + 1) // world
    a1, a2 = np.triu_indices(C5_NANTS, 1)
    nbl = len(a1)
    perm, _, rs, ant2 = kernels.canonical_baselines(a1, a2, C5_NANTS)
    a1t = torch.as_tensor(a1[perm], device=dev)
    a2t = torch.as_tensor(a2[perm], device=dev)
    gen = torch.Generator(device=dev)
    stats = {"iters": [], "err": 0.0, "res": 0.0, "sub_iters": 0}

    def batch_inputs(t0, nt):
        gen.manual_seed(1805550721 + t0)
        amp = torch.exp(0.1 * torch.randn((nt, C5_NANTS, C5_NCHAN), generator=gen, device=dev,
                                          dtype=torch.float64))
        ph = 0.1 * torch.randn((nt, C5_NANTS, C5_NCHAN), generator=gen, device=dev,
                               dtype=torch.float64)
        g = torch.polar(amp, ph)
        xb = (g[:, a1t, :] * torch.conj(g[:, a2t, :]))[..., None].contiguous()
        wb = torch.ones(xb.shape, dtype=torch.float64, device=dev)
        gain = torch.ones((nt, C5_NANTS, C5_NCHAN, 1, 1), dtype=torch.complex128, device=dev)
        gwt = torch.zeros((nt, C5_NANTS, C5_NCHAN, 1, 1), dtype=torch.float64, device=dev)
        return g, xb, wb, gain, gwt

    def one_pass(record):
        solve_s = 0.0
        for t0 in range(t_lo, t_hi, C5_BATCH):
            nt = min(C5_BATCH, t_hi - t0)
            g, xb, wb, gain, gwt = batch_inputs(t0, nt)
            torch.cuda.synchronize(dev)
            ta = time.perf_counter()
            res, used = kernels.solve_gains(xb, wb, gain, gwt, rs, ant2, mode=0, niter=200,
                                            tol=1e-6, phase_only=False)
            torch.cuda.synchronize(dev)
            solve_s += time.perf_counter() - ta
            if record:
                u = int(used.max())
                stats["iters"].append(u)
                stats["sub_iters"] += int(used.sum()) * C5_NCHAN  # used: per gain row
                est = gain[..., 0, 0]
                est = est * torch.conj(est[:, :1]) / torch.abs(est[:, :1])
                tru = g * torch.conj(g[:, :1]) / torch.abs(g[:, :1])
                stats["err"] = max(stats["err"], float(torch.max(torch.abs(est - tru))))
                stats["res"] = max(stats["res"], float(res.max()))
            del g, xb, wb, gain, gwt
        return solve_s

    steps = args.extra_steps if sub else args.steps
    warmup = min(args.warmup, 1) if sub else args.warmup
    for _ in range(warmup):
        one_pass(False)
    if world > 1:
        dist.barrier(device_ids=[dev.index])
    torch.cuda.synchronize(dev)
    elapsed = sum(one_pass(s == 0) for s in range(steps))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank != 0:
        return
    nsub = ntime * C5_NCHAN
    nsub_rank = (t_hi - t_lo) * C5_NCHAN
    gbs = 12 * nbl * stats["sub_iters"] / (elapsed / steps) / 1e9
    cpu = None
    if world == 1:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import ref_oracle as ro
        rng = np.random.default_rng(1805550721)
        gh = (rng.lognormal(0, 0.1, (2, C5_NANTS)) * np.exp(1j * rng.normal(0, 0.1, (2, C5_NANTS))))
        bl = np.stack([a1, a2], 1)
        tc0 = time.perf_counter()
        for s in range(2):
            xbh = (gh[s, a1] * np.conj(gh[s, a2]))[:, None, None]
            ro.stefcal_row(xbh, np.ones(xbh.shape), bl, C5_NANTS,
                           np.ones((C5_NANTS, 1, 1, 1), complex), np.zeros((C5_NANTS, 1, 1, 1)),
                           200, 1e-6, False)
        tc = (time.perf_counter() - tc0) / 2
        cpu = {"value": round(1.0 / tc, 3), "unit": "solves/s", "cores": 1, "kind": "port",
               "sample": f"oracle/ref_oracle.stefcal_row (numpy restatement of solvers.py:217-300), "
                         f"2 sub-solves of 512 stations, {tc:.2f} s each; C5 extrapolates to "
                         f"{nsub * tc / 3600:.1f} h"}
    line = {
        "metric": "StefCal solves/s (solve_gaintable, 512 stations x 256 chan x 1000 times)",
        "value": round(nsub / (elapsed / steps), 1), "unit": "solves/s",
        "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64 arithmetic, x/w fp32 storage (c128 gains)",
        "data": "synthetic: true gains lognormal(0, 0.1) x exp(i N(0, 0.1)) per (time, station, "
                "chan), x_b = g_a1 conj(g_a2), unit weights, generated on device per batch "
                "outside the timed segments",
        "config": {"workload": f"C5: 512 stations x 256 chan x {ntime} times = {nsub} solves "
                               "(B jones, scalar, niter 200, tol 1e-6)",
                   "solves": nsub, "solves_rank0": nsub_rank, "batch_rows": C5_BATCH,
                   "parallelism": f"times x{world}, no collective"},
        "solve_stats_rank0": {"iterations_max": max(stats["iters"]) if stats["iters"] else 0,
                              "max_gain_err": stats["err"], "max_residual": stats["res"]},
        "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "whole solve (k_fill + k_iter + k_residual)",
                     "note": "12 B per baseline per sub-solve iteration (SURVEY.md 8(d)) over the "
                             "timed solves, per-sub-solve iteration counts summed"},
        "cpu_baseline": cpu,
    }
    if sub:
        return line
    print(json.dumps(line), flush=True)


def _cu_split_streams(dev, mode):
    """Two HIP streams on disjoint CU masks (hipExtStreamCreateWithCUMask),
    wrapped as torch ExternalStreams."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (ncu + 31) // 32
    out = []
    for which in (0, 1):
        bits = [0] * words
        for c in range(ncu):
            if mode == "alt":
                take = c % 2 == which
            elif mode == "ovl":  # 3/4 of the CUs each, half of them shared
                take = c % 4 != (3 if which == 0 else 1)
            else:
                take = (c < ncu // 2) == (which == 0)
            if take:
                bits[c // 32] |= 1 << (c % 32)
        arr = (ctypes.c_uint32 * words)(*bits)
        st = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), arr)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {rc}")
        out.append(torch.cuda.ExternalStream(st.value, device=dev))
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 via torchrun")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    if args.config in ("c3", "c5"):
        (run_c3 if args.config == "c3" else run_c5)(args, world, rank, dev)
        if world > 1:
            dist.destroy_process_group()
        return
    if args.config == "c4":
        if args.emulate and world == 1:
            er, ew = (int(x) for x in args.emulate.split("/"))
            run_c4(args, ew, er, local, dev, emulated=True)
        else:
            run_c4(args, world, rank, local, dev)
        if world > 1:
            dist.destroy_process_group()
        return

    from ska_sdp_func_python_amd import kernels, parallel, simulation

    nchan_total = args.nchan * world
    chans = parallel.interleaved_channels(nchan_total, rank, world)
    obs = simulation.device_observation(args.ntimes, args.nchan, F_LO, F_HI, config="MID",
                                        seed=rank, device=dev, nchan_total=nchan_total,
                                        channels=chans)
    cell = 0.25 / obs["umax"]
    nvis_rank = obs["nrow"] * len(chans)
    out = torch.empty((args.npix, args.npix), dtype=torch.float64, device=dev)
    infos = []

    # two streams and two library scratch slots (SDP_HIP_SLOT1): step i runs on
    # stream i % 2, so step i+1's bucketing (memory-side atomics) overlaps
    # step i's gridding and FFTs; every step is still a complete invert with
    # its own image
    # (--cu-split, default 'alt': the two streams on disjoint halves of the CUs,
    # so one step's latency-bound bucketing and the other's gridding / FFT
    # share the chip by CU instead of by workgroup dispatch order; the serial
    # pass below runs on the default stream, every CU)
    pipe = args.pipeline
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)] if pipe else [None]
    if pipe and args.cu_split:
        try:
            streams = _cu_split_streams(dev, args.cu_split)
        except (OSError, AttributeError, RuntimeError) as e:  # (no CU-mask API: unmasked)
            print(f"bench: CU-masked streams unavailable ({e!r}); unmasked", file=sys.stderr)
            args.cu_split = ""
    outs = [out] + ([torch.empty_like(out)] if pipe else [])

    # the weight sum (ng.py:258) comes from the gridding call's count pass,
    # which reads the weights anyway (kernels.ms2dirty_vis, invert_ng's entry
    # point); SDP_BENCH_FUSED_SUMWT=0: bare ms2dirty + a separate torch sum
    fused_sw = os.environ.get("SDP_BENCH_FUSED_SUMWT", "1") != "0"

    def grid_fn_slot(slot):
        def fn(uvw, freq, vis, wgt, *a, **k):
            if fused_sw:
                r = kernels.ms2dirty_vis(uvw, freq, vis.unsqueeze(2), 0, wgt, None, None, *a,
                                         slot=slot, **k)
            else:
                r = kernels.ms2dirty(uvw, freq, vis, wgt, *a, slot=slot, **k)
            infos.append(r[1])
            return r
        return fn

    def step(i=0, pipelined=True):
        j = i % len(streams) if pipelined else 0

        def run():
            parallel.invert_sharded(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], args.npix,
                                    cell, EPS_REQUESTED, True, flip_uw=True, normalise=True,
                                    grid_fn=grid_fn_slot(j), out=outs[j], fused_sumwt=fused_sw)
        if streams[j] is None or not pipelined:  # (serial: the whole GPU, default stream)
            run()
        else:
            with torch.cuda.stream(streams[j]):
                run()

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local])
        torch.cuda.synchronize(dev)

    kernels.set_stage_timing(False)
    for i in range(max(args.warmup, 2 if pipe else 0)):
        step(i)
    barrier()

    def timed(pipelined):
        barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(i, pipelined)
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    elapsed = timed(pipe)
    # the gridder's launch duration: a serial pass (one stream) with stage
    # timing on -- the C ABI brackets k_grid with HIP events on its launch
    # stream, which synchronises the host after each call, so it is not the
    # timed (overlapped) loop
    kernels.set_stage_timing(True)
    infos.clear()
    elapsed_serial = timed(False)
    kernels.set_stage_timing(False)

    info = infos[-1]
    ms_step = elapsed / args.steps * 1e3
    value = nvis_rank * world / (elapsed / args.steps) / 1e6
    ms_grid = float(np.mean([i["ms_grid"] for i in infos]))
    launches = max(1, info["grid_launches"])
    alg_bytes = nvis_rank * (8 + 4 + 24.0 / len(chans)) + \
        info["nplanes"] * info["ngrid_x"] * info["ngrid_y"] * 8
    achieved = alg_bytes / launches / (ms_grid / launches * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic):
        with open(args.traffic) as f:
            traffic = json.load(f).get("bytes_per_launch")
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": (f"k_grid_mfma_pad<{info['support']},true>" if info.get("padded")
                       else f"k_grid_mfma<{info['support']},true> (sub-sorted cells)"),
            "kernel_ms": round(ms_grid / launches, 4),
            "alg_bytes_per_launch": int(alg_bytes / launches),
            # the gridder's work is fp32 MFMA (v_mfma_f32_16x16x4_f32): the
            # same kernel against the fp32 matrix peak (= the fp32 vector peak
            # on gfx950), 4 W^3 flops per visibility
            "compute": {"achieved": round(nvis_rank * 4 * info["support"] ** 3 / (ms_grid * 1e-3) / 1e12, 2),
                        "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(nvis_rank * 4 * info["support"] ** 3 / (ms_grid * 1e-3) / 1e12
                                      / FP32_PEAK_TFLOPS, 4)}}

    def guarded(fn, *a):
        """an auxiliary object of the line: its failure is recorded in the
        line instead of losing the headline measurement"""
        try:
            return fn(*a)
        except Exception as e:  # noqa: BLE001
            print(f"bench: {fn.__name__} failed: {e!r}", file=sys.stderr, flush=True)
            return {"error": repr(e)[:300]}

    api = None
    if rank == 0 and world == 1 and not args.no_api:
        api = guarded(api_rates, args, obs, cell)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_chans > 0:
        cpu = cpu_baseline(args, obs["umax"], nchan_total)

    extra = {}
    if world == 1 and not args.no_extra:
        r = guarded(c2_predict_and_fp64, args, obs, cell, dev, cpu)
        extra.update(r if "error" not in r else {"c2_predict": r})
        # the other configurations, each timed on its own (free the C2 inputs
        # first: the whole-band C4 needs ~250 GB of HBM)
        del obs
        out = None
        torch.cuda.synchronize(dev)
        kernels.release_workspace()
        torch.cuda.empty_cache()
        extra["c4_n1"] = guarded(run_c4, args, 1, 0, local, dev, False, True)
        kernels.release_workspace()
        torch.cuda.empty_cache()
        extra["c3"] = guarded(run_c3, args, 1, 0, dev, True)
        extra["c5"] = guarded(run_c5, args, 1, 0, dev, True)
        kernels.release_workspace()
        torch.cuda.empty_cache()

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mvis/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded SKA-MID-like layout, N(0,1) c64 vis, unit f32 weights, "
                    "generated on device)",
            "config": {"workload": "C2: SKA-MID 197 dishes, 64 chan x 100 times per GPU, "
                                   f"{args.npix}^2 image, {info['ngrid_x']}^2 w-stack grid",
                       "pipelined": ("consecutive inverts on two streams / library scratch "
                                     "slots: step i+1's bucketing under step i's gridding + "
                                     "FFT" + (f"; streams on disjoint CU masks ({args.cu_split})"
                                              if args.cu_split else "") if pipe else False),
                       "ms_per_step_serial": round(elapsed_serial / args.steps * 1e3, 3),
                       "value_serial": round(nvis_rank * world / (elapsed_serial / args.steps)
                                             / 1e6, 3),
                       "nvis_per_gpu": nvis_rank, "nchan_total": nchan_total,
                       "npix": args.npix, "cell_rad": cell, "support": info["support"],
                       "nplanes": info["nplanes"], "epsilon_requested": EPS_REQUESTED,
                       "parallelism": f"channel-sharded x{world}, 1 all-reduce"},
            "stages_ms": {k: round(float(np.mean([i[k] for i in infos])), 3)
                          for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "api": api,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
