"""Quick on-GPU parity + timing probe for the NUFFT pair (dev script)."""
import os, sys, time
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from ska_sdp_func_python_amd import kernels
import nufft_oracle as orc

rng = np.random.default_rng(1)
dev = torch.device("cuda:0")
nrow, nchan, npix = 400, 3, 64
freq = np.array([1.0e9, 1.1e9, 1.2e9])
umax = 2000.0
uvw = rng.uniform(-1, 1, (nrow, 3)) * umax * orc.C_LIGHT / freq.max()
uvw[:, 2] *= 0.5
pix = 0.45 / umax
ms = rng.normal(size=(nrow, nchan)) + 1j * rng.normal(size=(nrow, nchan))
wgt = rng.uniform(0.5, 1.5, (nrow, nchan))
T = lambda a, dt=None: torch.as_tensor(a, device=dev) if dt is None else torch.as_tensor(a, device=dev, dtype=dt)
for dow in (False, True):
    ex = orc.ms2dirty_exact(uvw, freq, ms, wgt.astype(np.float32), npix, npix, pix, pix, dow)
    for vdt in (torch.complex64, torch.complex128):
        out, info = kernels.ms2dirty(T(uvw), T(freq), T(ms, vdt), T(wgt, torch.float32), npix, npix, pix, pix, 1e-7, dow)
        d = out.cpu().numpy()
        err = np.sqrt(np.mean((d - ex) ** 2)) / np.sqrt(np.mean(ex ** 2))
        print("ms2dirty do_w=%d %s rel_rms=%.3e W=%d planes=%d" % (dow, vdt, err, info["support"], info["nplanes"]))
    # adjoint
    img = rng.normal(size=(npix, npix))
    exv = orc.dirty2ms_exact(uvw, freq, img, wgt.astype(np.float32), pix, pix, dow)
    v, info = kernels.dirty2ms(T(uvw), T(freq), T(img), T(wgt, torch.float32), pix, pix, 1e-7, dow, vis_dtype=torch.complex128)
    vv = v.cpu().numpy()
    err = np.sqrt(np.mean(np.abs(vv - exv) ** 2)) / np.sqrt(np.mean(np.abs(exv) ** 2))
    print("dirty2ms do_w=%d rel_rms=%.3e" % (dow, err))

# timing probe: medium-size random problem
nrow, nchan, npix = 200000, 64, 2048
freq = np.linspace(0.95e9, 1.76e9, nchan)
umax = 1e5
r = rng.uniform(0, 1, nrow) ** 2 * umax * orc.C_LIGHT / freq.max()
th = rng.uniform(0, 2 * np.pi, nrow)
uvw = np.stack([r * np.cos(th), r * np.sin(th), 0.3 * r * rng.normal(size=nrow)], 1)
pix = 0.25 / umax
uvw_t = T(uvw); f_t = T(freq)
vis_t = torch.randn(nrow, nchan, dtype=torch.complex64, device=dev)
w_t = torch.ones(nrow, nchan, dtype=torch.float32, device=dev)
kernels.set_stage_timing(True)
for it in range(3):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    out, info = kernels.ms2dirty(uvw_t, f_t, vis_t, w_t, npix, npix, pix, pix, 1e-7, True)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    print("ms2dirty %d vis npix %d: %.2f ms -> %.1f Mvis/s" % (nrow * nchan, npix, (t1 - t0) * 1e3, nrow * nchan / (t1 - t0) / 1e6), info)
for it in range(2):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    v, info = kernels.dirty2ms(uvw_t, f_t, out, w_t, pix, pix, 1e-7, True)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    print("dirty2ms: %.2f ms" % ((t1 - t0) * 1e3), info)
