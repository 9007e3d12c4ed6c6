import os, sys, time
sys.path.insert(0, "ska-sdp-func-python_amd")
import numpy as np, torch
from ska_sdp_func_python_amd import kernels, simulation
dev = torch.device("cuda:0")
obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, device=dev)
cell = 0.25 / obs["umax"]
img = torch.randn(4096, 4096, dtype=torch.float64, device=dev)
out = torch.empty_like(obs["vis"])
for mode in ("0", "1", "0", "1"):
    os.environ["SDP_HIP_PIPELINE"] = mode
    kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell, 1e-12, True, flip_uw=True, out=out)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(5):
        kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell, 1e-12, True, flip_uw=True, out=out)
    torch.cuda.synchronize(); t = (time.perf_counter() - t0) / 5
    print("predict pipeline=%s %.2f ms" % (mode, t * 1e3), flush=True)
