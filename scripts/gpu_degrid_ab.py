"""C2 predict: MFMA degridder (one-cell buckets) vs the register degridder
(SDP_HIP_MFMA_DEGRID=0): wall time, degridding stage time and the relative
RMS difference of the two visibility sets."""
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
img = torch.randn(4096, 4096, dtype=torch.float64, device=dev)
res = {}
outs = {}
for mode in ("1", "0", "1", "0"):
    os.environ["SDP_HIP_MFMA_DEGRID"] = mode
    out = torch.empty_like(obs["vis"])
    kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell, 1e-12, True,
                     flip_uw=True, out=out)
    kernels.set_stage_timing(True)
    infos = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        _, info = kernels.dirty2ms(obs["uvw"], obs["freq"], img, obs["wgt"], cell, cell, 1e-12,
                                   True, flip_uw=True, out=out)
        infos.append(info)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / 5
    kernels.set_stage_timing(False)
    outs[mode] = out
    g = sum(i["ms_grid"] for i in infos) / len(infos)
    p = sum(i["ms_prep"] for i in infos) / len(infos)
    res["mfma" if mode == "1" else "reg"] = {"ms": round(t * 1e3, 2), "ms_grid": round(g, 2),
                                            "ms_prep": round(p, 2), "bucket": infos[-1]["bucket"],
                                            "mvis_s": round(obs["vis"].numel() / t / 1e6, 1)}
    print(mode, res, flush=True)
d = (outs["1"] - outs["0"]).abs().pow(2).mean().sqrt() / outs["0"].abs().pow(2).mean().sqrt()
res["rel_rms_mfma_vs_reg"] = float(d)
print(json.dumps(res), flush=True)
