"""Dev probe: C4-geometry invert (SKA-LOW, 8192^2 image) stage timings under
different kernel knobs (env vars).  usage: gpu_sweep_c4.py KNOB v1,v2 [ntimes nchan]"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
import numpy as np, torch
from ska_sdp_func_python_amd import kernels, parallel, simulation

knob, vals = sys.argv[1], sys.argv[2].split(",")
ntimes = int(sys.argv[3]) if len(sys.argv) > 3 else 100
nchan = int(sys.argv[4]) if len(sys.argv) > 4 else 8
dev = torch.device("cuda:0")
chans = parallel.interleaved_channels(256, 0, 256 // nchan)
obs = simulation.device_observation(ntimes, nchan, 50e6, 350e6, config="LOW", device=dev,
                                    nchan_total=256, channels=chans)
cell = 0.25 / obs["umax"]
kernels.set_stage_timing(True)
for v in vals:
    os.environ[knob] = v
    res = []
    for it in range(3):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        img, info = kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], 8192, 8192,
                                     cell, cell, 1e-12, True, flip_uw=True)
        torch.cuda.synchronize(); t1 = time.perf_counter()
        if it > 0:
            res.append(((t1 - t0) * 1e3, info["ms_prep"], info["ms_grid"], info["ms_fft"]))
    m = np.mean(res, axis=0)
    print(json.dumps({knob: v, "wall_ms": round(m[0], 2), "prep": round(m[1], 2), "grid": round(m[2], 2),
                      "fft": round(m[3], 2), "nvis": obs["nrow"] * nchan}), flush=True)
