"""CPU analysis of the C2 bucketing (bench.py's SKA-MID layout, 64 channels x
100 times, 4096^2 image, 8192^2 grid, W = 8): records per 64 x 64-cell bin,
per cell, and the channel runs a range-based bucketing would store per bin
(profiles/r06_c2_bucket_stats.txt)."""
import sys, math, numpy as np
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))), "ska-sdp-func-python_amd"))
from ska_sdp_func_python_amd import simulation as sim
C = 299792458.0
fn, n_def, lat, dec_def = sim.CONFIGS["MID"]
en = fn(n_def, seed=1)
ha = np.linspace(-0.5, 0.5, 100) * 8.0 * math.pi / 12.0
uvw, _ = sim.observe(en, math.radians(lat), math.radians(dec_def), ha)
uvw = uvw.reshape(-1, 3)
freq = np.linspace(0.95e9, 1.76e9, 64)
umax = float(np.max(np.abs(uvw[:, :2]))) * freq.max() / C
npix = 4096; px = 0.25 / umax; ng = 8192; W = 8
lmax = (npix // 2) * px; r2 = min(2 * lmax * lmax, 1.0); tmax = 1 - math.sqrt(1 - r2)
dw = 1 / (2 * tmax)
s = freq / C
u = -uvw[:, 0:1] * s; v = uvw[:, 1:2] * s; w = -uvw[:, 2:3] * s
wmin, wmax = w.min(), w.max()
w0 = wmin - (0.5 * W - 0.5) * dw
a = u * px * ng; b = v * py if False else v * px * ng
fa = np.floor(a - 0.5 * W); fb = np.floor(b - 0.5 * W)
ic = (fa + 1 + ng // 2).astype(np.int64); jc = (fb + 1 + ng // 2).astype(np.int64)
pw = (w - w0) / dw
p0 = (np.floor(pw - 0.5 * W) + 1).astype(np.int64)
nrow, nch = ic.shape
print("nrow", nrow, "nvis", nrow * nch, "nps", p0.max() + 1, "ic range", ic.min(), ic.max())
binkey = (p0 * 200 + (ic >> 6)) * 200 + (jc >> 6)
# entries: runs of equal bin along channels per row
chg = np.ones_like(binkey, dtype=bool); chg[:, 1:] = binkey[:, 1:] != binkey[:, :-1]
nent = chg.sum(); print("entries", nent, "records/entry", nrow * nch / nent)
# entries for cell-level and 2x8 group level
cellkey = (p0 * 10000 + ic) * 10000 + jc
c2 = np.ones_like(cellkey, dtype=bool); c2[:, 1:] = cellkey[:, 1:] != cellkey[:, :-1]
print("cell runs", c2.sum())
bins, bc = np.unique(binkey, return_counts=True)
print("bins", len(bins), "records/bin: max", bc.max(), "median", np.median(bc), "p90", np.percentile(bc, 90))
order = np.argsort(-bc); cs = np.cumsum(bc[order]) / bc.sum()
print("top bins share:", [round(float(cs[k]), 3) for k in (0, 1, 4, 9, 49, 99)])
cells, cc = np.unique(cellkey, return_counts=True)
print("cells", len(cells), "records/cell max", cc.max(), "median", np.median(cc), "mean", cc.mean())
pad = ((cc + 3) // 4 * 4).sum(); print("padded", pad, pad / cc.sum())
for lim in (1, 2, 4, 8, 16, 64, 256, 4096):
    print(f"records in cells with <= {lim}:", round(float(cc[cc <= lim].sum() / cc.sum()), 4))
