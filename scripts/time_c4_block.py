"""Stage times of one C4 channel-block invert (32 of 256 SKA-LOW channels,
1.67 Gvis, 8192^2 image on a 16384^2 grid, 71 w planes): for A/Bs of the
plane-stage kernels (e.g. SDP_HIP_XFFT_FUSED=0/1) at the 16384-point x edge."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))

import torch  # noqa: E402

from ska_sdp_func_python_amd import kernels, simulation  # noqa: E402

dev = torch.device("cuda:0")
obs = simulation.device_observation(400, 32, 50e6, 350e6, config="LOW", device=dev,
                                    nchan_total=256, channels=list(range(224, 256)))
cell = 0.25 / obs["umax"]
kernels.set_stage_timing(True)
res = []
for _ in range(3):
    out, info = kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], 8192, 8192, cell,
                                 cell, 1e-7, True, flip_uw=True)
    res.append({k: round(float(info[k]), 2) for k in ("ms_prep", "ms_grid", "ms_fft", "ms_screen")})
torch.cuda.synchronize()
print(json.dumps({"fused": os.environ.get("SDP_HIP_XFFT_FUSED", "1"), "stages": res[1:],
                  "checksum": float(out.double().sum())}))
