"""ORACLE / TEST INFRASTRUCTURE ONLY -- ctypes front end of oracle/wgrid_cpu.c.

Used by tests/ (second checker of the HIP gridder) and by bench.py's
``cpu_baseline`` leg.  Never imported by the product package.
"""

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libwgrid_cpu.so")
_lib = None


def build():
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        lib = ctypes.CDLL(_SO)
        p = ctypes.c_void_p
        lib.wgrid_cpu_ms2dirty.argtypes = [p, p, ctypes.c_int, ctypes.c_int64, p, p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                           ctypes.c_double, ctypes.c_int, p, ctypes.c_int, p, p]
        lib.wgrid_cpu_ms2dirty.restype = ctypes.c_int
        lib.wgrid_cpu_dirty2ms.argtypes = [p, p, ctypes.c_int, ctypes.c_int64, p, p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                           ctypes.c_double, ctypes.c_int, p, ctypes.c_int, p, p]
        lib.wgrid_cpu_dirty2ms.restype = ctypes.c_int
        _lib = lib
    return _lib


def ms2dirty(uvw, freq, ms, wgt, npix_x, npix_y, pixsize_x, pixsize_y, epsilon=1e-7,
             do_wstacking=True, nthreads=0):
    """ducc0-convention ms2dirty on the host; returns (dirty [nx, ny], t_grid, t_fft)."""
    lib = load()
    uvw = np.ascontiguousarray(uvw, np.float64)
    freq = np.ascontiguousarray(freq, np.float64)
    nrow, nchan = uvw.shape[0], freq.shape[0]
    vis = None if ms is None else np.ascontiguousarray(ms, np.complex64)
    wt = None if wgt is None else np.ascontiguousarray(wgt, np.float32)
    out = np.zeros((npix_x, npix_y), np.float64)
    tg, tf = ctypes.c_double(), ctypes.c_double()
    ptr = lambda a: None if a is None else a.ctypes.data
    rc = lib.wgrid_cpu_ms2dirty(ptr(uvw), ptr(freq), nchan, nrow, ptr(vis), ptr(wt), npix_x, npix_y,
                                pixsize_x, pixsize_y, epsilon, int(bool(do_wstacking)), ptr(out),
                                int(nthreads), ctypes.byref(tg), ctypes.byref(tf))
    if rc != 0:
        raise ValueError("wgrid_cpu_ms2dirty failed (npix must be even)")
    return out, tg.value, tf.value


def dirty2ms(uvw, freq, dirty, wgt, pixsize_x, pixsize_y, epsilon=1e-7, do_wstacking=True,
             nthreads=0):
    """ducc0-convention dirty2ms on the host (the adjoint of ms2dirty above);
    dirty is [npix_x, npix_y]; returns (vis [nrow, nchan] complex128, t_degrid, t_fft)."""
    lib = load()
    uvw = np.ascontiguousarray(uvw, np.float64)
    freq = np.ascontiguousarray(freq, np.float64)
    dirty = np.ascontiguousarray(dirty, np.float64)
    nrow, nchan = uvw.shape[0], freq.shape[0]
    npix_x, npix_y = dirty.shape
    wt = None if wgt is None else np.ascontiguousarray(np.broadcast_to(wgt, (nrow, nchan)),
                                                       np.float32)
    out = np.zeros((nrow, nchan), np.complex128)
    tg, tf = ctypes.c_double(), ctypes.c_double()
    ptr = lambda a: None if a is None else a.ctypes.data
    rc = lib.wgrid_cpu_dirty2ms(ptr(uvw), ptr(freq), nchan, nrow, ptr(dirty), ptr(wt), npix_x,
                                npix_y, pixsize_x, pixsize_y, epsilon, int(bool(do_wstacking)),
                                ptr(out), int(nthreads), ctypes.byref(tg), ctypes.byref(tf))
    if rc != 0:
        raise ValueError("wgrid_cpu_dirty2ms failed (npix must be even)")
    return out, tg.value, tf.value
