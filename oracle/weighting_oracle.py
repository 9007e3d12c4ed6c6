"""CPU restatement of the reference's imaging-weight path (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module, as the checker; the product path is the HIP kernels in
ska-sdp-func-python_amd/csrc/weighting.hip.

Vectorised numpy restatement of
  * grid_visibility_weight_to_griddata  src/ska_sdp_func_python/grid_data/gridding.py:258-334
  * griddata_visibility_reweight        gridding.py:362-499
  * spatial_mapping (no cf)             gridding.py:142-157, via
    convolution_mapping_visibility      gridding.py:33-57
  * taper_visibility_gaussian           src/ska_sdp_func_python/imaging/weighting.py:71-101
  * taper_visibility_tukey              weighting.py:104-136 (+ tukey_filter,
                                        src/ska_sdp_func_python/util/array_functions.py:85-99)
Pinned by tests/golden/weight_*.npz (made by running the reference's own
function bodies, tests/golden/make_golden.py).

Arrays are flat over rows: uvw [nrow, 3] metres, weights [nrow, nchan, npol].
``wcs`` is ((crval_u, cdelt_u, crpix_u), (crval_v, cdelt_v, crpix_v)) of the
GridData's UU/VV axes; pixel = (world - crval) / cdelt + crpix - 1 (origin 0).
"""

import numpy as np

C_M_S = 299792458.0


def _pix(world, ax):
    crval, cdelt, crpix = ax
    return np.round((world - crval) / cdelt + crpix - 1).astype(np.int64)


def mapping(uvw, freq, chan, wcs):
    """gridding.py:49-57 + :148-157: nearest cell of (u, v) and of (-u, -v)."""
    k = freq[chan] / C_M_S
    u = np.nan_to_num(uvw[:, 0] * k)
    v = np.nan_to_num(uvw[:, 1] * k)
    return _pix(u, wcs[0]), _pix(v, wcs[1]), _pix(-u, wcs[0]), _pix(-v, wcs[1])


def _ingrid(pu, pv, puc, pvc, ny, nx):
    return ((pv >= 0) & (pv < ny) & (pu >= 0) & (pu < nx)
            & (pvc >= 0) & (pvc < ny) & (puc >= 0) & (puc < nx))


def grid_weights(uvw, freq, fwt, vis_to_im, wcs, g_nchan, ny, nx):
    """gridding.py:258-334: both the sample and its conjugate cell get the
    flagged weight; rows whose cell or conjugate cell is off the grid are
    skipped.  Returns (grid f64 [g_nchan, npol, ny, nx], sumwt, nskipped)."""
    nrow, nchan, npol = fwt.shape
    grid = np.zeros((g_nchan, npol, ny, nx))
    sumwt = np.zeros((g_nchan, npol))
    nskipped = 0
    for ch in range(nchan):
        ic = vis_to_im[ch]
        pu, pv, puc, pvc = mapping(uvw, freq, ch, wcs)
        ok = _ingrid(pu, pv, puc, pvc, ny, nx)
        nskipped += int((~ok).sum()) * npol
        for p in range(npol):
            w = fwt[ok, ch, p]
            np.add.at(grid[ic, p], (pv[ok], pu[ok]), w)
            np.add.at(grid[ic, p], (pvc[ok], puc[ok]), w)
            sumwt[ic, p] += 2.0 * w.sum()
    return grid, sumwt, nskipped


def reweight(uvw, freq, fwt, fimw, vis_to_im, wcs, grid, weighting="uniform",
             robustness=0.0, sumwt=None):
    """gridding.py:362-499.  ``fwt`` / ``fimw`` are the flagged weight and
    flagged imaging weight; returns the new imaging weight."""
    assert weighting in ("natural", "uniform", "robust"), f"Weighting {weighting} not supported"
    nrow, nchan, npol = fwt.shape
    out = np.array(fimw, dtype=float, copy=True)
    if weighting == "robust":
        sumlocwt = np.sum(grid ** 2)
        total = np.sum(fwt) * 2 if sumwt is None else np.sum(sumwt)
        f2 = (5.0 * np.power(10.0, -robustness)) ** 2 * total / sumlocwt
    _, _, ny, nx = grid.shape
    for ch in range(nchan):
        ic = vis_to_im[ch]
        pu, pv, puc, pvc = mapping(uvw, freq, ch, wcs)
        ok = _ingrid(pu, pv, puc, pvc, ny, nx)
        for p in range(npol):
            g = np.zeros(nrow)
            g[ok] = grid[ic, p, pv[ok], pu[ok]]
            col = out[:, ch, p]
            col[~ok] = 0.0
            pos = ok & (g > 0.0)
            if weighting == "uniform":
                col[pos] = fwt[pos, ch, p] / g[pos]
            else:
                col[pos] = fwt[pos, ch, p] / (1 + f2 * g[pos])
            col[ok & (g <= 0.0)] = 0.0
    return out


def taper_gaussian(uvw, freq, fimw, beam):
    """weighting.py:71-101: fimw * exp(-pi^2 beam^2 / (4 ln 2) |uv|^2)."""
    scale = np.pi ** 2 * beam ** 2 / (4.0 * np.log(2.0))
    out = np.empty_like(fimw)
    for ch, f in enumerate(freq):
        wave = C_M_S / f
        uvdistsq = (uvw[:, 0] ** 2 + uvw[:, 1] ** 2) / wave ** 2
        out[:, ch, :] = fimw[:, ch, :] * np.exp(-scale * uvdistsq)[:, None]
    return out


def tukey_filter(x, r):
    """array_functions.py:85-99, vectorised."""
    y = np.ones_like(x)
    lo = (x >= 0.0) & (x < r / 2.0)
    hi = (x >= 1 - r / 2.0) & (x <= 1.0) & ~lo
    y[lo] = 0.5 * (1.0 + np.cos(2.0 * np.pi * (x[lo] - r / 2.0) / r))
    y[hi] = 0.5 * (1.0 + np.cos(2.0 * np.pi * (x[hi] - 1 + r / 2.0) / r))
    return y


def taper_tukey(uvw, freq, fimw, tukey=0.1):
    """weighting.py:104-136: radius normalised by its maximum per channel."""
    out = np.empty_like(fimw)
    for ch, f in enumerate(freq):
        wave = C_M_S / f
        uvdist = np.sqrt(uvw[:, 0] ** 2 + uvw[:, 1] ** 2) / wave
        uvdist = uvdist / np.max(uvdist)
        out[:, ch, :] = fimw[:, ch, :] * tukey_filter(uvdist, tukey)[:, None]
    return out
