"""C2 predict (dirty2ms, epsilon 1e-7 -> the fp32 NUFFT, W = 8) timing for A/B
runs of library builds (SDP_HIP_LIB_OVERRIDE selects the build): wall time
per call, degridding stage time, and a checksum of the visibilities."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ska-sdp-func-python_amd"))
import torch  # noqa: E402
from ska_sdp_func_python_amd import kernels, simulation  # noqa: E402

dev = torch.device("cuda:0")
obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, device=dev)
cell = 0.25 / obs["umax"]
g = torch.Generator(device=dev)
g.manual_seed(5)
img = torch.randn(4096, 4096, dtype=torch.float64, device=dev, generator=g)
out = torch.empty_like(obs["vis"])
for _ in range(2):
    kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell, 1e-7, True,
                     flip_uw=True, out=out)
kernels.set_stage_timing(True)
infos = []
torch.cuda.synchronize()
t0 = time.perf_counter()
n = 10
for _ in range(n):
    _, info = kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell, 1e-7, True,
                               flip_uw=True, out=out)
    infos.append(info)
torch.cuda.synchronize()
t = (time.perf_counter() - t0) / n
kernels.set_stage_timing(False)
print(json.dumps({"lib": os.environ.get("SDP_HIP_LIB_OVERRIDE", "in-tree"),
                  "ms": round(t * 1e3, 3), "mvis_s": round(out.numel() / t / 1e6, 1),
                  "ms_grid": round(sum(i["ms_grid"] for i in infos) / n, 3),
                  "ms_prep": round(sum(i["ms_prep"] for i in infos) / n, 3),
                  "ms_fft": round(sum(i["ms_fft"] for i in infos) / n, 3),
                  "checksum": float(torch.sum(torch.abs(out.to(torch.complex128))))}))
