"""Tensor-level wrappers over the C ABI (device buffers are torch tensors).

These are the thin host shims between the reference-shaped Python API
(imaging/, calibration/, grid_data/) and libska_sdp_hip.so.  They validate
shapes, dtypes and devices, pass raw device pointers + element strides, and
enqueue on torch's current HIP stream.  Nothing here computes on the CPU.
"""

import ctypes

import torch

from . import _lib

_DT_CODE = {
    torch.complex64: _lib.SDP_HIP_C64,
    torch.complex128: _lib.SDP_HIP_C128,
    torch.float32: _lib.SDP_HIP_F32,
    torch.float64: _lib.SDP_HIP_F64,
}


def _on_gpu(t, name):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a device (HIP) tensor")
    return t


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _check_uvw(uvw):
    _on_gpu(uvw, "uvw")
    if uvw.dtype != torch.float64 or uvw.dim() != 2 or uvw.shape[1] != 3 or uvw.stride(1) != 1:
        raise ValueError("uvw must be float64 [nrow, 3] with unit column stride")


def ms2dirty(uvw, freq, vis, wgt, npix_x, npix_y, pixsize_x, pixsize_y,
             epsilon=1e-7, do_wstacking=True, flip_uw=False, out=None,
             out_strides=None, accumulate=False):
    """ducc0.wgridder.ms2dirty semantics on device.

    uvw [nrow,3] f64, freq [nchan] f64, vis [nrow,nchan] c64/c128 (or None
    for unit visibilities), wgt [nrow,nchan] f32 (or None).  Returns the
    f64 dirty image [npix_x, npix_y] (or writes ``out`` with
    ``out_strides`` = (stride_x, stride_y) in elements) and an info dict.
    """
    _check_uvw(uvw)
    dev = uvw.device
    freq = _on_gpu(freq, "freq").to(torch.float64).contiguous()
    nrow, nchan = uvw.shape[0], freq.shape[0]
    if vis is not None:
        _on_gpu(vis, "vis")
        if vis.dtype not in (torch.complex64, torch.complex128) or tuple(vis.shape) != (nrow, nchan):
            raise ValueError("vis must be complex [nrow, nchan]")
    if wgt is not None:
        _on_gpu(wgt, "wgt")
        if wgt.dtype != torch.float32 or tuple(wgt.shape) != (nrow, nchan):
            raise ValueError("wgt must be float32 [nrow, nchan]")
    if out is None:
        out = torch.empty((npix_x, npix_y), dtype=torch.float64, device=dev)
        out_strides = (npix_y, 1)
    elif out_strides is None:
        out_strides = out.stride()
    _on_gpu(out, "out")
    if out.dtype != torch.float64:
        raise ValueError("dirty output must be float64")
    flags = (_lib.SDP_HIP_FLIP_UW if flip_uw else 0) | (_lib.SDP_HIP_ACCUMULATE if accumulate else 0)
    info = _lib.WGridInfo()
    _lib.call(
        "sdp_hip_ms2dirty",
        _ptr(uvw), uvw.stride(0), _ptr(freq), nchan, nrow,
        _ptr(vis), _DT_CODE[vis.dtype] if vis is not None else _lib.SDP_HIP_C64,
        vis.stride(0) if vis is not None else 0, vis.stride(1) if vis is not None else 0,
        _ptr(wgt), wgt.stride(0) if wgt is not None else 0, wgt.stride(1) if wgt is not None else 0,
        int(npix_x), int(npix_y), float(pixsize_x), float(pixsize_y), float(epsilon),
        int(bool(do_wstacking)), flags,
        _ptr(out), int(out_strides[0]), int(out_strides[1]),
        _stream(dev), ctypes.byref(info))
    return out, info.as_dict()


def dirty2ms(uvw, freq, dirty, wgt, pixsize_x, pixsize_y, epsilon=1e-7,
             do_wstacking=True, flip_uw=False, out=None, dirty_strides=None,
             npix=None, accumulate=False, vis_dtype=torch.complex64):
    """ducc0.wgridder.dirty2ms semantics on device; returns vis [nrow,nchan]."""
    _check_uvw(uvw)
    dev = uvw.device
    freq = _on_gpu(freq, "freq").to(torch.float64).contiguous()
    nrow, nchan = uvw.shape[0], freq.shape[0]
    _on_gpu(dirty, "dirty")
    if dirty.dtype != torch.float64:
        raise ValueError("dirty must be float64")
    if npix is None:
        npix_x, npix_y = dirty.shape[-2], dirty.shape[-1]
    else:
        npix_x, npix_y = npix
    if dirty_strides is None:
        dirty_strides = dirty.stride()[-2:]
    if wgt is not None:
        _on_gpu(wgt, "wgt")
        if wgt.dtype != torch.float32 or tuple(wgt.shape) != (nrow, nchan):
            raise ValueError("wgt must be float32 [nrow, nchan]")
    if out is None:
        out = torch.empty((nrow, nchan), dtype=vis_dtype, device=dev)
    _on_gpu(out, "vis out")
    if out.dtype not in (torch.complex64, torch.complex128) or tuple(out.shape) != (nrow, nchan):
        raise ValueError("vis out must be complex [nrow, nchan]")
    flags = (_lib.SDP_HIP_FLIP_UW if flip_uw else 0) | (_lib.SDP_HIP_ACCUMULATE if accumulate else 0)
    info = _lib.WGridInfo()
    _lib.call(
        "sdp_hip_dirty2ms",
        _ptr(uvw), uvw.stride(0), _ptr(freq), nchan, nrow,
        _ptr(dirty), int(dirty_strides[0]), int(dirty_strides[1]), int(npix_x), int(npix_y),
        float(pixsize_x), float(pixsize_y),
        _ptr(wgt), wgt.stride(0) if wgt is not None else 0, wgt.stride(1) if wgt is not None else 0,
        float(epsilon), int(bool(do_wstacking)), flags,
        _ptr(out), _DT_CODE[out.dtype], out.stride(0), out.stride(1),
        _stream(dev), ctypes.byref(info))
    return out, info.as_dict()


def set_stage_timing(enable):
    _lib.load().sdp_hip_set_stage_timing(int(bool(enable)))


def release_workspace():
    _lib.call("sdp_hip_release_workspace")
