"""C2 invert_ng shapes beyond the single-pol MFS bench line:
1 pol vs 4 pols (independent buckets vs one shared bucketing), and the
64-channel cube (one image per channel), timed through kernels.ms2dirty_vis
exactly as invert_ng calls it.  Prints one JSON line per case."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
import torch
from ska_sdp_func_python_amd import kernels, simulation

dev = torch.device("cuda:0")
obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, device=dev)
nrow, nchan, npix = obs["nrow"], 64, 4096
cell = 0.25 / obs["umax"]
g = torch.Generator(device=dev)
g.manual_seed(5)
vis4 = torch.randn((nrow, nchan, 4), generator=g, device=dev, dtype=torch.complex64)
wgt4 = torch.ones((nrow, nchan, 4), device=dev, dtype=torch.float32)
flags = torch.zeros((nrow, nchan, 4), device=dev, dtype=torch.int8)
out = torch.zeros((4, npix, npix), dtype=torch.float64, device=dev)
uvw, freq = obs["uvw"], obs["freq"]


def call(pol, chans, keep=False, reuse=False):
    kernels.ms2dirty_vis(uvw, freq[chans], vis4[:, chans, :], pol, wgt4[:, chans, pol], flags[:, chans, :],
                         None, npix, npix, cell, cell, 1e-7, True, flip_uw=True, out=out[pol],
                         accumulate=True, keep_buckets=keep, reuse_buckets=reuse)


def timed(name, fn, reps=3, nvis=nrow * nchan):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    print(json.dumps({"case": name, "ms": round(ms, 2), "Mvis_s_per_pol": round(nvis / ms / 1e3, 1)}),
          flush=True)
    return ms


mfs = slice(0, nchan)
t1 = timed("mfs 1 pol", lambda: call(0, mfs))
t4i = timed("mfs 4 pol, independent bucketing", lambda: [call(p, mfs) for p in range(4)], nvis=4 * nrow * nchan)
t4s = timed("mfs 4 pol, shared bucketing",
            lambda: [call(p, mfs, keep=p == 0, reuse=p > 0) for p in range(4)], nvis=4 * nrow * nchan)
print(json.dumps({"ratio_4pol_shared_over_1pol": round(t4s / t1, 2),
                  "ratio_4pol_independent_over_1pol": round(t4i / t1, 2)}), flush=True)
timed("cube 64 chan x 1 pol", lambda: [call(0, slice(c, c + 1)) for c in range(nchan)], reps=1)
timed("cube 64 chan x 4 pol, shared per channel",
      lambda: [call(p, slice(c, c + 1), keep=p == 0, reuse=p > 0) for c in range(nchan) for p in range(4)],
      reps=1, nvis=4 * nrow * nchan)
