"""C2 invert prep time only (for count-pass experiments)."""
import json, os, sys, time
sys.path.insert(0, "/root/repo/ska-sdp-func-python_amd")
import numpy as np, torch
from ska_sdp_func_python_amd import kernels, simulation
dev = torch.device("cuda:0")
obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, config="MID", seed=0, device=dev)
cell = 0.25 / obs["umax"]
kernels.set_stage_timing(True)
ps = []
for i in range(5):
    _, info = kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], 4096, 4096,
                               cell, cell, 1e-12, True, flip_uw=True)
    ps.append(info["ms_prep"])
print(os.environ.get("SDP_HIP_CEXP", "0"), json.dumps({"ms_prep": round(float(np.median(ps[1:])), 3)}))
