"""Dev probe: gridding time vs uv distribution and ablations."""
import os, sys, time
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
from ska_sdp_func_python_amd import kernels
C = 299792458.0
rng = np.random.default_rng(1)
dev = torch.device("cuda:0")
nrow, nchan, npix = 200000, 64, 2048
freq = np.linspace(0.95e9, 1.76e9, nchan)
umax = 1e5
pix = 0.25 / umax
kernels.set_stage_timing(True)
vis_t = torch.randn(nrow, nchan, dtype=torch.complex64, device=dev)
w_t = torch.ones(nrow, nchan, dtype=torch.float32, device=dev)
f_t = torch.as_tensor(freq, device=dev)
for dist in ("uniform", "square"):
    u01 = rng.uniform(0, 1, nrow)
    r = (np.sqrt(u01) if dist == "uniform" else u01 ** 2) * umax * C / freq.max()
    th = rng.uniform(0, 2 * np.pi, nrow)
    uvw = np.stack([r * np.cos(th), r * np.sin(th), 0.3 * r * rng.normal(size=nrow)], 1)
    uvw_t = torch.as_tensor(uvw, device=dev)
    for mode in ("x",):
        for dow in (False, True):
            best = 1e9
            for it in range(3):
                torch.cuda.synchronize(); t0 = time.perf_counter()
                out, info = kernels.ms2dirty(uvw_t, f_t, vis_t, w_t, npix, npix, pix, pix, 1e-7, dow)
                torch.cuda.synchronize(); t1 = time.perf_counter()
                best = min(best, t1 - t0)
            v2, i2 = kernels.dirty2ms(uvw_t, f_t, out, w_t, pix, pix, 1e-7, dow)
            torch.cuda.synchronize(); t0 = time.perf_counter()
            v2, i2 = kernels.dirty2ms(uvw_t, f_t, out, w_t, pix, pix, 1e-7, dow)
            torch.cuda.synchronize(); t2 = time.perf_counter() - t0
            print(f"{dist:8s} PB={mode} predict {t2*1e3:8.2f} ms degrid {i2['ms_grid']:8.2f}")
            print(f"{dist:8s} PB={mode} do_w={int(dow)} total {best*1e3:8.2f} ms grid {info['ms_grid']:8.2f} ms items {info['nitems']} planes {info['nplanes']}", flush=True)
