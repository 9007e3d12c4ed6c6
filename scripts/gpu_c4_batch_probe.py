"""Dev probe: per-batch stage times of one C4 channel block streamed through
kernels.ms2dirty_batch with different batch counts (SKA-LOW, 8192^2 image)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
import numpy as np, torch
from ska_sdp_func_python_amd import kernels, simulation

lo, hi = int(sys.argv[1]), int(sys.argv[2])
nbs = [int(x) for x in sys.argv[3].split(",")]
dev = torch.device("cuda:0")
freqs = np.linspace(50e6, 350e6, 256)
obs = simulation.device_observation(400, 1, 50e6, 350e6, config="LOW", seed=0, device=dev,
                                    nchan_total=256, channels=[lo])
uvw, nrow = obs["uvw"], obs["nrow"]
cell = 0.25 / obs["umax"]
freq = torch.as_tensor(freqs[lo:hi], device=dev)
g = torch.Generator(device=dev)
g.manual_seed(3)
vis = torch.randn((nrow, hi - lo), generator=g, device=dev, dtype=torch.complex64)
out = torch.zeros((8192, 8192), dtype=torch.float64, device=dev)
kernels.set_stage_timing(True)
salts = sys.argv[4].split(",") if len(sys.argv) > 4 else [os.environ.get("SDP_HIP_SALT", "8")]
for salt, nb in [(s_, n_) for s_ in salts for n_ in nbs]:
    os.environ["SDP_HIP_SALT"] = salt
    cuts = [(hi - lo) * i // nb for i in range(nb + 1)]
    blocks = list(zip(cuts[:-1], cuts[1:]))
    b = kernels.merge_bounds(*[kernels.uvw_bounds(uvw, freq[a:e]) for a, e in blocks])
    for rep in range(2):
        infos = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, (a, e) in enumerate(blocks):
            _, info = kernels.ms2dirty_batch(uvw, freq[a:e], vis[:, a:e], None, 8192, 8192, cell, cell, b,
                                             first=i == 0, last=i == nb - 1, epsilon=1e-12,
                                             do_wstacking=True, flip_uw=True, out=out,
                                             out_strides=(1, 8192), accumulate=True)
            infos.append({k: round(info[k], 1) for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")})
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"block": [lo, hi], "salt": salt, "batches": nb, "ms": round(ms, 1), "per_batch": infos,
                      "nplanes": info["nplanes"], "nitems": info["nitems"]}), flush=True)
