"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

CPU restatement of the predict/invert NUFFT pair that the reference binds
through ``ducc0.wgridder`` (ducc0 0.27.0, ``poetry.lock:305-306``; call sites
``src/ska_sdp_func_python/imaging/ng.py:99``, ``:117``, ``:240``, ``:271``).

ducc0 is a third-party C++ library that is *not* vendored under
/root/reference and cannot be installed here, so parity at this boundary is
anchored on the exact direct sums that ducc0 approximates to ``epsilon``
(SURVEY.md Appendix A):

    ms2dirty:  dirty[x, y] = sum_k wgt_k Re{ ms_k exp(+2 pi i (u l_x + v m_y - w (n - 1))) } [/ n]
    dirty2ms:  ms_k        = wgt_k sum_{x,y} dirty[x, y] exp(-2 pi i (u l_x + v m_y - w (n - 1))) [/ n]

with ``l_x = (x - nx//2) * pixsize_x``, ``m_y = (y - ny//2) * pixsize_y``,
uvw in wavelengths (``uvw * f / c``), ``1/n`` and the w term only when
``do_wstacking`` is true, and pixels beyond the horizon set to zero.  This is
the *ducc0* (caller-facing) convention: RASCIL's ``invert_ng`` negates u and w
and transposes the result (``ng.py:210-213``, ``:257``).

Also here: ``wgrid_ms2dirty`` / ``wgrid_dirty2ms``, a small numpy restatement of
the w-gridding algorithm (ES kernel, oversampled grid, w planes, grid
correction) that the HIP path implements; it is used to validate the
algorithm's error budget against the exact sums.  Parity status: the exact
sums are the definition ducc0 approximates; no ducc0 output exists here, so the
ducc0 boundary is "parity unpinned" beyond those semantics.
"""

import numpy as np

C_LIGHT = 299792458.0


def _lm_grid(npix_x, npix_y, pixsize_x, pixsize_y):
    x = (np.arange(npix_x) - npix_x // 2) * pixsize_x
    y = (np.arange(npix_y) - npix_y // 2) * pixsize_y
    l2 = x[:, None] ** 2
    m2 = y[None, :] ** 2
    r2 = l2 + m2
    inside = r2 < 1.0
    nm1 = np.where(inside, -r2 / (np.sqrt(np.where(inside, 1.0 - r2, 1.0)) + 1.0), 0.0)
    return x, y, nm1, inside


def ms2dirty_exact(uvw, freq, ms, wgt, npix_x, npix_y, pixsize_x, pixsize_y,
                   do_wstacking):
    """Exact adjoint NUFFT (ducc0 convention).  uvw [nrow,3] m, freq [nchan],
    ms [nrow,nchan] complex, wgt [nrow,nchan] or None.  Returns f64 [nx,ny]."""
    uvw = np.asarray(uvw, dtype=np.float64)
    freq = np.asarray(freq, dtype=np.float64)
    ms = np.asarray(ms, dtype=np.complex128)
    if wgt is None:
        wgt = np.ones(ms.shape)
    scale = freq[None, :] / C_LIGHT
    u = (uvw[:, 0:1] * scale).ravel()
    v = (uvw[:, 1:2] * scale).ravel()
    w = (uvw[:, 2:3] * scale).ravel()
    c = (ms * wgt).ravel()
    keep = c != 0
    u, v, w, c = u[keep], v[keep], w[keep], c[keep]
    lx, my, nm1, inside = _lm_grid(npix_x, npix_y, pixsize_x, pixsize_y)
    dirty = np.zeros((npix_x, npix_y))
    # blocked over x rows to bound memory
    for ix in range(npix_x):
        ph = u[:, None] * lx[ix] + v[:, None] * my[None, :]
        if do_wstacking:
            ph = ph - w[:, None] * nm1[ix][None, :]
        ph = 2.0 * np.pi * ph
        dirty[ix] = (c.real[:, None] * np.cos(ph) - c.imag[:, None] * np.sin(ph)).sum(axis=0)
    if do_wstacking:
        dirty = np.where(inside, dirty / (nm1 + 1.0), 0.0)
    return dirty


def dirty2ms_exact(uvw, freq, dirty, wgt, pixsize_x, pixsize_y, do_wstacking):
    """Exact forward NUFFT (ducc0 convention).  Returns complex [nrow,nchan]."""
    uvw = np.asarray(uvw, dtype=np.float64)
    freq = np.asarray(freq, dtype=np.float64)
    dirty = np.asarray(dirty, dtype=np.float64)
    npix_x, npix_y = dirty.shape
    lx, my, nm1, inside = _lm_grid(npix_x, npix_y, pixsize_x, pixsize_y)
    img = dirty.copy()
    if do_wstacking:
        img = np.where(inside, img / (nm1 + 1.0), 0.0)
    nrow, nchan = uvw.shape[0], freq.shape[0]
    out = np.zeros((nrow, nchan), dtype=np.complex128)
    L = np.broadcast_to(lx[:, None], img.shape).ravel()
    M = np.broadcast_to(my[None, :], img.shape).ravel()
    N = nm1.ravel()
    I = img.ravel()
    for ch in range(nchan):
        s = freq[ch] / C_LIGHT
        u = uvw[:, 0] * s
        v = uvw[:, 1] * s
        w = uvw[:, 2] * s
        for r0 in range(0, nrow, 256):
            r1 = min(nrow, r0 + 256)
            ph = u[r0:r1, None] * L[None] + v[r0:r1, None] * M[None]
            if do_wstacking:
                ph = ph - w[r0:r1, None] * N[None]
            out[r0:r1, ch] = (I[None] * np.exp(-2j * np.pi * ph)).sum(axis=1)
    if wgt is not None:
        out = out * wgt
    return out


# ---------------------------------------------------------------------------
# w-gridding restatement (algorithm check, small sizes only)
# ---------------------------------------------------------------------------

def kernel_params(epsilon):
    """Support W and ES shape beta for oversampling sigma = 2 (FINUFFT rule)."""
    eps = max(float(epsilon), 1.0e-7)
    W = int(np.ceil(-np.log10(eps / 10.0)))
    W = min(max(W, 2), 8)
    return W, 2.30 * W


def es_kernel(t, W, beta):
    x = 2.0 * np.asarray(t, dtype=np.float64) / W
    y = 1.0 - x * x
    return np.where(y > 0.0, np.exp(beta * (np.sqrt(np.maximum(y, 0.0)) - 1.0)), 0.0)


def es_fourier(xi, W, beta, nquad=128):
    """Phi(xi) = int_{-W/2}^{W/2} phi(t) cos(2 pi t xi) dt (Gauss-Legendre)."""
    z, wq = np.polynomial.legendre.leggauss(nquad)
    t = 0.25 * W * (z + 1.0)          # nodes on [0, W/2]
    wt = 0.25 * W * wq
    phi = es_kernel(t, W, beta)
    xi = np.asarray(xi, dtype=np.float64)
    return 2.0 * (wt * phi * np.cos(2.0 * np.pi * np.multiply.outer(xi, t))).sum(axis=-1)


def wgrid_geometry(uvw_lambda_w, npix_x, npix_y, pixsize_x, pixsize_y, do_wstacking, W):
    ngx = 2 * npix_x
    ngy = 2 * npix_y
    if not do_wstacking:
        return dict(ngx=ngx, ngy=ngy, nplanes=1, w0=0.0, dw=1.0, s0=0.0)
    lmax = (npix_x // 2) * pixsize_x
    mmax = (npix_y // 2) * pixsize_y
    r2 = min(lmax * lmax + mmax * mmax, 1.0)
    tmax = 1.0 - np.sqrt(1.0 - r2)
    wmin, wmax = float(np.min(uvw_lambda_w)), float(np.max(uvw_lambda_w))
    s0 = 0.5 * tmax
    dw = 1.0 / (2.0 * tmax) if tmax > 0 else 1.0
    w0 = wmin - (0.5 * W - 0.5) * dw
    pwmax = (wmax - w0) / dw
    nplanes = int(np.floor(pwmax - 0.5 * W)) + 1 + W
    return dict(ngx=ngx, ngy=ngy, nplanes=nplanes, w0=w0, dw=dw, s0=s0)


def wgrid_ms2dirty(uvw, freq, ms, wgt, npix_x, npix_y, pixsize_x, pixsize_y,
                   do_wstacking, epsilon=1e-7):
    """Numpy restatement of the w-gridding adjoint the HIP path implements."""
    W, beta = kernel_params(epsilon)
    scale = np.asarray(freq)[None, :] / C_LIGHT
    u = (uvw[:, 0:1] * scale).ravel()
    v = (uvw[:, 1:2] * scale).ravel()
    w = (uvw[:, 2:3] * scale).ravel()
    c = (np.asarray(ms, np.complex128) * (1.0 if wgt is None else wgt)).ravel()
    g = wgrid_geometry(w, npix_x, npix_y, pixsize_x, pixsize_y, do_wstacking, W)
    ngx, ngy, npl = g["ngx"], g["ngy"], g["nplanes"]
    grid = np.zeros((npl, ngx, ngy), dtype=np.complex128)
    a = u * pixsize_x * ngx
    b = v * pixsize_y * ngy
    i0 = np.floor(a - 0.5 * W).astype(np.int64) + 1
    j0 = np.floor(b - 0.5 * W).astype(np.int64) + 1
    if do_wstacking:
        c = c * np.exp(2j * np.pi * w * g["s0"])
        pw = (w - g["w0"]) / g["dw"]
        p0 = np.floor(pw - 0.5 * W).astype(np.int64) + 1
    for k in range(W):
        ku = es_kernel(i0 + k - a, W, beta)
        gi = (i0 + k + ngx // 2) % ngx
        for kk in range(W):
            kv = es_kernel(j0 + kk - b, W, beta)
            gj = (j0 + kk + ngy // 2) % ngy
            if do_wstacking:
                for kw in range(W):
                    wk = es_kernel(p0 + kw - pw, W, beta)
                    np.add.at(grid, (p0 + kw, gi, gj), c * ku * kv * wk)
            else:
                np.add.at(grid, (0, gi, gj), c * ku * kv)
    H = np.fft.ifft2(grid, axes=(1, 2)) * (ngx * ngy)
    X = np.arange(npix_x) - npix_x // 2
    Y = np.arange(npix_y) - npix_y // 2
    sub = H[:, X[:, None] % ngx, Y[None, :] % ngy]
    sign = np.where(((X[:, None] + Y[None, :]) & 1) == 1, -1.0, 1.0)
    lx, my, nm1, inside = _lm_grid(npix_x, npix_y, pixsize_x, pixsize_y)
    corr = 1.0 / (es_fourier(np.abs(X) / ngx, W, beta)[:, None]
                  * es_fourier(np.abs(Y) / ngy, W, beta)[None, :])
    if do_wstacking:
        s = -nm1 - g["s0"]
        wp = g["w0"] + np.arange(npl) * g["dw"]
        acc = (sub * np.exp(2j * np.pi * wp[:, None, None] * s[None])).sum(axis=0).real
        corr = corr / es_fourier(np.abs(g["dw"] * s), W, beta)
        dirty = np.where(inside, acc * sign * corr / (nm1 + 1.0), 0.0)
    else:
        dirty = sub[0].real * sign * corr
    return dirty
