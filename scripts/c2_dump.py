"""One C2 invert (bench.py's workload) with the library selected by
SDP_HIP_LIB_OVERRIDE, dirty image saved to --out (.npy); with --ref, the
relative RMS difference against a saved image and against an fp64 (eps 1e-12)
invert of the same inputs is printed: the A/B precision check for gridder
variants."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))

import torch  # noqa: E402

from ska_sdp_func_python_amd import kernels, simulation  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", required=True)
ap.add_argument("--ref", default=None)
ap.add_argument("--exact", action="store_true", help="also an eps 1e-12 run as the exact result")
ap.add_argument("--predict", action="store_true", help="dirty2ms of a random image instead")
a = ap.parse_args()
dev = torch.device("cuda:0")
npix = 4096
obs = simulation.device_observation(100, 64, 0.95e9, 1.76e9, config="MID", seed=0, device=dev)
cell = 0.25 / obs["umax"]

def run(eps):
    if a.predict:
        gen = torch.Generator(device=dev).manual_seed(3)
        dirty = torch.randn(npix, npix, dtype=torch.float64, device=dev, generator=gen)
        v = kernels.dirty2ms(obs["uvw"], obs["freq"], dirty, obs["wgt"], cell, cell, eps, True,
                             flip_uw=True)[0].reshape(-1)[::7].cpu().numpy()
        return np.stack([v.real, v.imag]).astype(np.float64)  # (every 7th visibility)
    return kernels.ms2dirty(obs["uvw"], obs["freq"], obs["vis"], obs["wgt"], npix, npix, cell, cell,
                            eps, True, flip_uw=True)[0].cpu().numpy()


img = run(1e-7)
np.save(a.out, img)
res = {"lib": os.environ.get("SDP_HIP_LIB_OVERRIDE", "in-tree"), "rms": float(np.sqrt(np.mean(img ** 2)))}
if a.exact:
    ex = run(1e-12)
    np.save(a.out.replace(".npy", "_exact.npy"), ex)
if a.ref:
    ref = np.load(a.ref)
    res["rel_vs_ref"] = float(np.sqrt(np.mean((img - ref) ** 2) / np.mean(ref ** 2)))
    exf = a.ref.replace(".npy", "_exact.npy")
    if os.path.exists(exf):
        ex = np.load(exf)
        res["rel_vs_exact"] = float(np.sqrt(np.mean((img - ex) ** 2) / np.mean(ex ** 2)))
        res["ref_rel_vs_exact"] = float(np.sqrt(np.mean((ref - ex) ** 2) / np.mean(ex ** 2)))
print(json.dumps(res))
