"""ORACLE / TEST INFRASTRUCTURE ONLY -- ctypes front end of oracle/wgrid_cpu.c.

Used by tests/ (full-size checker of the HIP gridder) and by bench.py's
``cpu_baseline`` leg.  Never imported by the product package.

``precision="single"``: fp32 taps and grid, W <= 8 (epsilon floored at 1e-7),
the arithmetic the HIP path performs.  ``precision="double"``: fp64 taps, grid
and visibilities, W <= 16 (epsilon 1e-12 -> W = 13): the reference's ducc0
call with ``double_precision_accumulation=True``
(src/ska_sdp_func_python/imaging/ng.py:240-256).
"""

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libwgrid_cpu.so")
_lib = None
_PREC = {"single": 0, "double": 1}


def build():
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        lib = ctypes.CDLL(_SO)
        p, i, i64, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
        lib.wgrid_cpu_ms2dirty.argtypes = [p, p, i, i64, p, i, p, i, i, i, d, d, d, i, i, p, i,
                                           p, p, p, p]
        lib.wgrid_cpu_ms2dirty.restype = i
        lib.wgrid_cpu_dirty2ms.argtypes = [p, p, i, i64, p, p, i, i, i, d, d, d, i, i, p, i,
                                           p, p, p, p]
        lib.wgrid_cpu_dirty2ms.restype = i
        lib.wgrid_cpu_exact_pixels.argtypes = [p, p, i, i64, p, i, p, i, i, i, d, d, i, i, p, p,
                                               p, i]
        lib.wgrid_cpu_exact_pixels.restype = i
        lib.wgrid_cpu_exact_rows.argtypes = [p, p, i, i, p, p, i, i, d, d, i, p, i]
        lib.wgrid_cpu_exact_rows.restype = i
        _lib = lib
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def _vis_arg(ms):
    if ms is None:
        return None, 0
    ms = np.asarray(ms)
    if ms.dtype == np.complex128:
        return np.ascontiguousarray(ms), 1
    return np.ascontiguousarray(ms, np.complex64), 0


def _wgt_arg(wgt, shape=None):
    if wgt is None:
        return None, 0
    wgt = np.asarray(wgt)
    if shape is not None:
        wgt = np.broadcast_to(wgt, shape)
    if wgt.dtype == np.float64:
        return np.ascontiguousarray(wgt), 1
    return np.ascontiguousarray(wgt, np.float32), 0


def ms2dirty(uvw, freq, ms, wgt, npix_x, npix_y, pixsize_x, pixsize_y, epsilon=1e-7,
             do_wstacking=True, nthreads=0, precision="single", info=None):
    """ducc0-convention ms2dirty on the host; returns (dirty [nx, ny], t_grid, t_fft).
    ms may be complex64 or complex128, wgt float32 or float64 (read as given).
    `info`, if a dict, receives the support W and the plane count."""
    lib = load()
    uvw = np.ascontiguousarray(uvw, np.float64)
    freq = np.ascontiguousarray(freq, np.float64)
    nrow, nchan = uvw.shape[0], freq.shape[0]
    vis, vis64 = _vis_arg(ms)
    wt, wt64 = _wgt_arg(wgt)
    out = np.zeros((npix_x, npix_y), np.float64)
    tg, tf = ctypes.c_double(), ctypes.c_double()
    sup, npl = ctypes.c_int(), ctypes.c_int()
    rc = lib.wgrid_cpu_ms2dirty(_ptr(uvw), _ptr(freq), nchan, nrow, _ptr(vis), vis64, _ptr(wt),
                                wt64, npix_x, npix_y, pixsize_x, pixsize_y, epsilon,
                                int(bool(do_wstacking)), _PREC[precision], _ptr(out),
                                int(nthreads), ctypes.byref(tg), ctypes.byref(tf),
                                ctypes.byref(sup), ctypes.byref(npl))
    if rc != 0:
        raise ValueError(f"wgrid_cpu_ms2dirty failed ({rc}: npix must be even, nvis < 2^32)")
    if info is not None:
        info.update(support=sup.value, nplanes=npl.value)
    return out, tg.value, tf.value


def dirty2ms(uvw, freq, dirty, wgt, pixsize_x, pixsize_y, epsilon=1e-7, do_wstacking=True,
             nthreads=0, precision="single", info=None):
    """ducc0-convention dirty2ms on the host (the adjoint of ms2dirty above);
    dirty is [npix_x, npix_y]; returns (vis [nrow, nchan] complex128, t_degrid, t_fft)."""
    lib = load()
    uvw = np.ascontiguousarray(uvw, np.float64)
    freq = np.ascontiguousarray(freq, np.float64)
    dirty = np.ascontiguousarray(dirty, np.float64)
    nrow, nchan = uvw.shape[0], freq.shape[0]
    npix_x, npix_y = dirty.shape
    wt, wt64 = _wgt_arg(wgt, (nrow, nchan))
    out = np.zeros((nrow, nchan), np.complex128)
    tg, tf = ctypes.c_double(), ctypes.c_double()
    sup, npl = ctypes.c_int(), ctypes.c_int()
    rc = lib.wgrid_cpu_dirty2ms(_ptr(uvw), _ptr(freq), nchan, nrow, _ptr(dirty), _ptr(wt), wt64,
                                npix_x, npix_y, pixsize_x, pixsize_y, epsilon,
                                int(bool(do_wstacking)), _PREC[precision], _ptr(out),
                                int(nthreads), ctypes.byref(tg), ctypes.byref(tf),
                                ctypes.byref(sup), ctypes.byref(npl))
    if rc != 0:
        raise ValueError("wgrid_cpu_dirty2ms failed (npix must be even)")
    if info is not None:
        info.update(support=sup.value, nplanes=npl.value)
    return out, tg.value, tf.value


def exact_pixels(uvw, freq, ms, wgt, npix_x, npix_y, pixsize_x, pixsize_y, do_wstacking,
                 px, py, nthreads=0):
    """Exact ms2dirty (ducc0 convention, nufft_oracle.ms2dirty_exact) at the
    pixels (px[i], py[i]); returns f64 [len(px)]."""
    lib = load()
    uvw = np.ascontiguousarray(uvw, np.float64)
    freq = np.ascontiguousarray(freq, np.float64)
    nrow, nchan = uvw.shape[0], freq.shape[0]
    vis, vis64 = _vis_arg(ms)
    wt, wt64 = _wgt_arg(wgt)
    px = np.ascontiguousarray(px, np.int32)
    py = np.ascontiguousarray(py, np.int32)
    out = np.zeros(px.shape[0], np.float64)
    lib.wgrid_cpu_exact_pixels(_ptr(uvw), _ptr(freq), nchan, nrow, _ptr(vis), vis64, _ptr(wt),
                               wt64, npix_x, npix_y, pixsize_x, pixsize_y,
                               int(bool(do_wstacking)), px.shape[0], _ptr(px), _ptr(py),
                               _ptr(out), int(nthreads))
    return out


def exact_rows(uvw, freq, dirty, rows, pixsize_x, pixsize_y, do_wstacking, nthreads=0):
    """Exact dirty2ms (ducc0 convention, unit weights) of the listed rows;
    returns complex128 [len(rows), nchan]."""
    lib = load()
    uvw = np.ascontiguousarray(uvw, np.float64)
    freq = np.ascontiguousarray(freq, np.float64)
    dirty = np.ascontiguousarray(dirty, np.float64)
    rows = np.ascontiguousarray(rows, np.int64)
    nchan = freq.shape[0]
    out = np.zeros((rows.shape[0], nchan), np.complex128)
    lib.wgrid_cpu_exact_rows(_ptr(uvw), _ptr(freq), nchan, rows.shape[0], _ptr(rows),
                             _ptr(dirty), dirty.shape[0], dirty.shape[1], pixsize_x, pixsize_y,
                             int(bool(do_wstacking)), _ptr(out), int(nthreads))
    return out
