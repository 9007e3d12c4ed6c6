"""ctypes binding of libska_sdp_hip.so (the C ABI declared in include/ska_sdp_hip.h).

The product path has exactly one backend: the hand-written HIP kernels in this
library.  If the shared object is missing or no GPU is visible, every compute
entry point raises -- there is deliberately no CPU fallback.
"""

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# SDP_HIP_LIB_OVERRIDE: load another build of the same C ABI (kernel-variant
# experiments, scripts/build_variants.sh); the default is the in-tree build.
LIB_PATH = os.environ.get("SDP_HIP_LIB_OVERRIDE") or os.path.join(_HERE, "_lib", "libska_sdp_hip.so")

SDP_HIP_OK = 0
SDP_HIP_ERR_INVALID_ARG = 1
SDP_HIP_ERR_RUNTIME = 2
SDP_HIP_ERR_NO_DEVICE = 3
SDP_HIP_ERR_MEMORY = 4

SDP_HIP_F32 = 1
SDP_HIP_F64 = 2
SDP_HIP_C64 = 3
SDP_HIP_C128 = 4

SDP_HIP_FLIP_UW = 1
SDP_HIP_ACCUMULATE = 2
SDP_HIP_BATCH_FIRST = 4
SDP_HIP_BATCH_LAST = 8
SDP_HIP_KEEP_BUCKETS = 16
SDP_HIP_REUSE_BUCKETS = 32
SDP_HIP_FP32 = 64
SDP_HIP_W_SLAB = 128
SDP_HIP_SLOT1 = 256

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_dbl = ctypes.c_double
c_vp = ctypes.c_void_p
c_u32 = ctypes.c_uint
c_size = ctypes.c_size_t
c_char_p = ctypes.c_char_p


class WGridInfo(ctypes.Structure):
    _fields_ = [
        ("support", c_int),
        ("beta", c_dbl),
        ("ngrid_x", c_int),
        ("ngrid_y", c_int),
        ("nplanes", c_int),
        ("w0", c_dbl),
        ("dw", c_dbl),
        ("nvis_used", c_i64),
        ("nitems", c_i64),
        ("plane_chunk", c_int),
        ("ms_prep", ctypes.c_float),
        ("ms_grid", ctypes.c_float),
        ("ms_fft", ctypes.c_float),
        ("ms_screen", ctypes.c_float),
        ("bucket", c_int),
        ("grid_launches", c_int),
        ("padded", c_int),
        ("fp64", c_int),
        ("tiled", c_int),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# (symbol, argtypes) for every entry point declared in include/ska_sdp_hip.h
_ERR = [c_char_p, c_size]
SIGNATURES = {
    "sdp_hip_version": [],
    "sdp_hip_device_count": [ctypes.POINTER(c_int)] + _ERR,
    "sdp_hip_release_workspace": _ERR,
    "sdp_hip_set_stage_timing": [c_int],
    "sdp_hip_ms2dirty": [
        c_vp, c_i64, c_vp, c_int, c_i64,          # uvw, stride, freq, nchan, nrow
        c_vp, c_int, c_i64, c_i64,                # vis, dtype, strides
        c_vp, c_int, c_i64, c_i64,                # wgt, dtype (f32 / f64), strides
        c_int, c_int, c_dbl, c_dbl, c_dbl, c_int, c_u32,
        c_vp, c_i64, c_i64,                       # dirty, strides
        c_vp, ctypes.POINTER(WGridInfo)] + _ERR,
    "sdp_hip_ms2dirty_batch": [
        c_vp, c_i64, c_vp, c_int, c_i64,          # uvw, stride, freq, nchan, nrow
        c_vp, c_int, c_i64, c_i64,                # vis, dtype, strides
        c_vp, c_int, c_i64, c_i64,                # wgt, dtype (f32 / f64), strides
        c_int, c_int, c_dbl, c_dbl, c_dbl, c_int, c_u32,
        c_vp,                                     # bounds (host, 6 doubles; 8 with W_SLAB)
        c_vp, c_i64, c_i64,                       # dirty, strides
        c_vp, ctypes.POINTER(WGridInfo)] + _ERR,
    "sdp_hip_wstack_layout": [
        c_vp, c_int, c_int, c_dbl, c_dbl, c_dbl, c_int, c_u32,  # bounds, geometry, eps, do_w, flags
        ctypes.POINTER(WGridInfo)] + _ERR,
    "sdp_hip_ms2dirty_vis": [
        c_vp, c_i64, c_vp, c_int, c_i64,          # uvw, stride, freq, nchan, nrow
        c_vp, c_int, c_i64, c_i64, c_i64, c_int,  # vis, dtype, row/chan/pol strides, npol_vis
        c_vp,                                     # pol_coeff (host doubles) or NULL
        c_vp, c_int, c_i64, c_i64,                # wgt, dtype, strides
        c_vp, c_int, c_i64, c_i64, c_i64, c_int,  # flags, bytes, strides, pol
        c_int, c_int, c_dbl, c_dbl, c_dbl, c_int, c_u32,
        c_vp, c_i64, c_i64, c_vp,                 # dirty, strides, sumwt
        c_vp,                                     # shift_lmn (host doubles) or NULL
        c_vp, ctypes.POINTER(WGridInfo)] + _ERR,
    "sdp_hip_ms2dirty_vis_pols": [
        c_vp, c_i64, c_vp, c_int, c_i64,          # uvw, stride, freq, nchan, nrow
        c_vp, c_int, c_i64, c_i64, c_i64, c_int,  # vis, dtype, row/chan/pol strides, npol_vis
        c_vp, c_int,                              # pol_coeff (host doubles) or NULL, npol_img
        c_vp, c_int, c_i64, c_i64, c_i64,         # wgt, dtype, row/chan/pol strides
        c_vp, c_int, c_i64, c_i64, c_i64,         # flags, bytes, strides
        c_int, c_int, c_dbl, c_dbl, c_dbl, c_int, c_u32,
        c_vp, c_i64, c_i64, c_i64,                # dirty, x / y / pol strides
        c_vp, c_i64,                              # sumwt, its pol stride
        c_vp,                                     # shift_lmn (host doubles) or NULL
        c_vp, ctypes.POINTER(WGridInfo)] + _ERR,
    "sdp_hip_ms2dirty_vis_batch": [
        c_vp, c_i64, c_vp, c_int, c_i64,          # uvw, stride, freq, nchan, nrow
        c_vp, c_int, c_i64, c_i64, c_i64, c_int,  # vis, dtype, row/chan/pol strides, npol_vis
        c_vp,                                     # pol_coeff (host doubles) or NULL
        c_vp, c_int, c_i64, c_i64,                # wgt, dtype, strides
        c_vp, c_int, c_i64, c_i64, c_i64, c_int,  # flags, bytes, strides, pol
        c_int, c_int, c_dbl, c_dbl, c_dbl, c_int, c_u32,
        c_vp,                                     # bounds (host, 6 doubles)
        c_vp, c_i64, c_i64, c_vp,                 # dirty, strides, sumwt
        c_vp,                                     # shift_lmn (host doubles) or NULL
        c_vp, ctypes.POINTER(WGridInfo)] + _ERR,
    "sdp_hip_dirty2ms": [
        c_vp, c_i64, c_vp, c_int, c_i64,
        c_vp, c_i64, c_i64, c_int, c_int, c_dbl, c_dbl,
        c_vp, c_int, c_i64, c_i64,                # wgt, dtype (f32 / f64), strides
        c_dbl, c_int, c_u32,
        c_vp, c_int, c_i64, c_i64,
        c_vp, ctypes.POINTER(WGridInfo)] + _ERR,
    "sdp_hip_dirty2ms_vis": [
        c_vp, c_i64, c_vp, c_int, c_i64,          # uvw, stride, freq, nchan, nrow
        c_vp, c_i64, c_i64, c_int, c_int, c_dbl, c_dbl,
        c_dbl, c_int, c_u32,
        c_vp, c_int, c_i64, c_i64, c_i64, c_int,  # vis, dtype, strides, npol_vis
        c_vp,                                     # pol_coeff (host doubles) or NULL
        c_vp,                                     # shift_lmn (host doubles) or NULL
        c_vp, ctypes.POINTER(WGridInfo)] + _ERR,
    "sdp_hip_dirty2ms_vis_pols": [
        c_vp, c_i64, c_vp, c_int, c_i64,          # uvw, stride, freq, nchan, nrow
        c_vp, c_i64, c_i64, c_i64, c_int,         # dirty, x / y / pol strides, npol_img
        c_int, c_int, c_dbl, c_dbl,
        c_dbl, c_int, c_u32,
        c_vp, c_int, c_i64, c_i64, c_i64, c_int,  # vis, dtype, strides, npol_vis
        c_vp,                                     # pol_coeff [npol_img][npol_vis] or NULL
        c_vp,                                     # shift_lmn (host doubles) or NULL
        c_vp, ctypes.POINTER(WGridInfo)] + _ERR,
    "sdp_hip_dft_point_v00": [
        c_int, c_vp, c_vp, c_int, c_int, c_i64, c_int, c_vp, c_vp, c_int, c_vp] + _ERR,
    "sdp_hip_dft_point_metres": [
        c_int, c_vp, c_vp, c_int, c_int, c_i64, c_int, c_vp, c_vp, c_vp, c_int,
        c_vp] + _ERR,
    "sdp_hip_grid_cf": [
        c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
        c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_int, c_int,
        c_int, c_vp, c_vp, c_vp] + _ERR,
    "sdp_hip_degrid_cf": [
        c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
        c_int, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp,
        c_vp, c_vp] + _ERR,
    "sdp_hip_solve_gains": [
        c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp,
        c_vp, c_vp, c_int, c_dbl, c_int, c_int, c_dbl, c_vp] + _ERR,
    "sdp_hip_point_sums": [
        c_i64, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp,
        c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp] + _ERR,
    "sdp_hip_divide_vis": [
        c_i64, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp] + _ERR,
    "sdp_hip_apply_gains": [
        c_i64, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp,
        c_vp, c_int, c_int, c_int, c_int, c_int, c_vp] + _ERR,
    "sdp_hip_grid_weights": [
        c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int,
        c_int, c_vp, c_vp, c_vp] + _ERR,
    "sdp_hip_reweight": [
        c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int,
        c_int, c_int, c_dbl, c_vp, c_int, c_vp, c_vp] + _ERR,
    "sdp_hip_taper": [
        c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_dbl, c_vp, c_vp] + _ERR,
}

_lock = threading.Lock()
_lib = None


class HipLibraryError(RuntimeError):
    """Raised when the native library is missing or no GPU is available."""


def load():
    """Load (once) and return the ctypes handle; raise if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise HipLibraryError(
                f"{LIB_PATH} not built: run __graft_entry__.build() "
                "(there is no CPU fallback for the HIP path)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = argtypes
            fn.restype = c_int
        _lib = lib
        return lib


def exported_symbols():
    lib = load()
    return [name for name in SIGNATURES if hasattr(lib, name)]


def errbuf():
    return ctypes.create_string_buffer(1024)


def check(status, buf):
    if status == SDP_HIP_OK:
        return
    msg = buf.value.decode(errors="replace") if buf is not None else ""
    if status == SDP_HIP_ERR_INVALID_ARG:
        raise ValueError(msg)
    if status == SDP_HIP_ERR_MEMORY:
        raise MemoryError(msg)
    raise RuntimeError(msg or f"libska_sdp_hip status {status}")


def call(name, *args):
    fn = getattr(load(), name)
    buf = errbuf()
    status = fn(*args, buf, ctypes.sizeof(buf))
    check(status, buf)
