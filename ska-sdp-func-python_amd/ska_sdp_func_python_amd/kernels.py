"""Tensor-level wrappers over the C ABI (device buffers are torch tensors).

These are the thin host shims between the reference-shaped Python API
(imaging/, calibration/, grid_data/) and libska_sdp_hip.so.  They validate
shapes, dtypes and devices, pass raw device pointers + element strides, and
enqueue on torch's current HIP stream.  Nothing here computes on the CPU.
"""

import ctypes
import logging

import torch

from . import _lib

log = logging.getLogger("func-python-logger")

# The w-stacking NUFFT has two precisions.  epsilon >= 1e-7: fp32 taps and
# uv planes with fp64 coordinates, phases and image accumulation (W <= 8;
# measured on the full C2 workload against the fp64 W = 13 oracle: 9.1e-7
# invert / 8.1e-7 predict relative RMS, tests/test_gpu_fullsize.py).
# epsilon < 1e-7 -- the reference's default 1e-12, which it asks of ducc0
# with double_precision_accumulation (imaging/ng.py:178, :240-256) -- runs
# the fp64 NUFFT (W = ceil(-log10(epsilon/10)) in [9, 16], c128 planes, Z2Z
# FFTs).  precision="fp32" (per call, or set_precision("fp32") for the
# process) keeps such requests on the fp32 path at its floor instead, said so
# once per process.
EPS_FLOOR = 1e-7
_PRECISION = "auto"
_eps_warned = False


def set_precision(mode):
    """Process default for the NUFFT precision: "auto" (fp64 below epsilon
    1e-7) or "fp32" (the fp32 NUFFT at its floor for every epsilon)."""
    global _PRECISION
    if mode not in ("auto", "fp32"):
        raise ValueError("precision must be 'auto' or 'fp32'")
    _PRECISION = mode


def is_fp64(epsilon, precision=None):
    """True when a NUFFT call at `epsilon` runs the fp64 path."""
    mode = precision or _PRECISION
    return float(epsilon) < EPS_FLOOR and mode == "auto"


def _prec_bits(epsilon, precision=None):
    """Flag bits of a NUFFT call for `epsilon` under `precision`."""
    global _eps_warned
    mode = precision or _PRECISION
    if mode not in ("auto", "fp32"):
        raise ValueError("precision must be 'auto' or 'fp32'")
    if float(epsilon) >= EPS_FLOOR or mode == "auto":
        return 0
    if not _eps_warned:
        _eps_warned = True
        log.warning("epsilon %.1e requested with precision='fp32': the HIP w-stacking NUFFT "
                    "runs in fp32 at its floor epsilon %.0e (support W = 8); measured "
                    "dirty-image error vs an fp64 epsilon=1e-12 reference ~1e-6 relative RMS",
                    float(epsilon), EPS_FLOOR)
    return _lib.SDP_HIP_FP32


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


def _alloc(shape, dtype, dev, may_release=True):
    """torch.empty on the device; when the caching allocator cannot serve it
    because the library's workspace holds the memory (cached w planes and
    records of an earlier large call), the workspace is released and the
    allocation retried once (the w planes are re-made on the next call).
    ``may_release=False`` (a batched invert past its first batch, whose
    resident planes hold the earlier batches' work) re-raises instead."""
    try:
        return torch.empty(shape, dtype=dtype, device=dev)
    except torch.OutOfMemoryError:
        if not may_release:
            raise
        release_workspace()
        torch.cuda.empty_cache()
        return torch.empty(shape, dtype=dtype, device=dev)


def _check_wgt(wgt, nrow, nchan):
    """ducc0 takes f64 weights; f32 (the bench's) and f64 are both read in place."""
    if wgt is None:
        return
    _on_gpu(wgt, "wgt")
    if wgt.dtype not in (torch.float32, torch.float64) or tuple(wgt.shape) != (nrow, nchan):
        raise ValueError("wgt must be float32 or float64 [nrow, nchan]")


def _wgt_args(wgt):
    if wgt is None:
        return (_ptr(None), _lib.SDP_HIP_F32, 0, 0)
    return (_ptr(wgt), _DT_CODE[wgt.dtype], wgt.stride(0), wgt.stride(1))


def _check_uvw(uvw):
    _on_gpu(uvw, "uvw")
    if uvw.dtype != torch.float64 or uvw.dim() != 2 or uvw.shape[1] != 3 or uvw.stride(1) != 1:
        raise ValueError("uvw must be float64 [nrow, 3] with unit column stride")


def ms2dirty(uvw, freq, vis, wgt, npix_x, npix_y, pixsize_x, pixsize_y,
             epsilon=1e-7, do_wstacking=True, flip_uw=False, out=None,
             out_strides=None, accumulate=False, precision=None, slot=0):
    """ducc0.wgridder.ms2dirty semantics on device.

    uvw [nrow,3] f64, freq [nchan] f64, vis [nrow,nchan] c64/c128 (or None
    for unit visibilities), wgt [nrow,nchan] f32 (or None).  Returns the
    f64 dirty image [npix_x, npix_y] (or writes ``out`` with
    ``out_strides`` = (stride_x, stride_y) in elements) and an info dict.
    ``slot=1`` uses the library's second scratch set (SDP_HIP_SLOT1): calls
    alternated between two streams and slots overlap on the device.
    """
    pbits = _prec_bits(epsilon, precision)
    _check_uvw(uvw)
    dev = uvw.device
    freq = _on_gpu(freq, "freq").to(torch.float64).contiguous()
    nrow, nchan = uvw.shape[0], freq.shape[0]
    if vis is not None:
        _on_gpu(vis, "vis")
        if vis.dtype not in (torch.complex64, torch.complex128) or tuple(vis.shape) != (nrow, nchan):
            raise ValueError("vis must be complex [nrow, nchan]")
    _check_wgt(wgt, nrow, nchan)
    if out is None:
        out = _alloc((npix_x, npix_y), torch.float64, dev)
        out_strides = (npix_y, 1)
    elif out_strides is None:
        out_strides = out.stride()
    _on_gpu(out, "out")
    if out.dtype != torch.float64:
        raise ValueError("dirty output must be float64")
    flags = ((_lib.SDP_HIP_FLIP_UW if flip_uw else 0) | (_lib.SDP_HIP_ACCUMULATE if accumulate else 0)
             | (_lib.SDP_HIP_SLOT1 if slot else 0) | pbits)
    info = _lib.WGridInfo()
    _lib.call(
        "sdp_hip_ms2dirty",
        _ptr(uvw), uvw.stride(0), _ptr(freq), nchan, nrow,
        _ptr(vis), _DT_CODE[vis.dtype] if vis is not None else _lib.SDP_HIP_C64,
        vis.stride(0) if vis is not None else 0, vis.stride(1) if vis is not None else 0,
        *_wgt_args(wgt),
        int(npix_x), int(npix_y), float(pixsize_x), float(pixsize_y), float(epsilon),
        int(bool(do_wstacking)), flags,
        _ptr(out), int(out_strides[0]), int(out_strides[1]),
        _stream(dev), ctypes.byref(info))
    return out, info.as_dict()


def uvw_bounds(uvw, freq):
    """Host {min w, max w, max|u|, max|v|, min f, max f} of device arrays uvw
    [nrow, 3] (metres) and freq: one batch's contribution to the bounds of
    an ms2dirty_batch sequence (combine with merge_bounds)."""
    _check_uvw(uvw)
    b = torch.stack([uvw[:, 2].min(), uvw[:, 2].max(), uvw[:, 0].abs().max(),
                     uvw[:, 1].abs().max(), freq.min().double(), freq.max().double()])
    return [float(x) for x in b.cpu()]


def merge_bounds(*bs):
    return [min(b[0] for b in bs), max(b[1] for b in bs), max(b[2] for b in bs),
            max(b[3] for b in bs), min(b[4] for b in bs), max(b[5] for b in bs)]


def wstack_layout(bounds, npix_x, npix_y, pixsize_x, pixsize_y, epsilon=1e-7, do_wstacking=True,
                  flip_uw=False, precision=None):
    """The w-plane layout an ms2dirty_batch sequence with these ``bounds``
    uses (sdp_hip_wstack_layout, no device work): dict with support, nplanes,
    w0, dw and ``nps`` = the first-plane count a w-slab partition splits."""
    if len(bounds) != 6:
        raise ValueError("bounds: {wmin, wmax, umax, vmax, fmin, fmax}")
    bbuf = (ctypes.c_double * 6)(*[float(x) for x in bounds])
    flags = (_lib.SDP_HIP_FLIP_UW if flip_uw else 0) | _prec_bits(epsilon, precision)
    info = _lib.WGridInfo()
    _lib.call("sdp_hip_wstack_layout", ctypes.cast(bbuf, ctypes.c_void_p), int(npix_x),
              int(npix_y), float(pixsize_x), float(pixsize_y), float(epsilon),
              int(bool(do_wstacking)), flags, ctypes.byref(info))
    d = info.as_dict()
    d["nps"] = d["nplanes"] - d["support"] + 1 if d["nplanes"] > 1 else 1
    return d


def ms2dirty_batch(uvw, freq, vis, wgt, npix_x, npix_y, pixsize_x, pixsize_y, bounds,
                   first, last, epsilon=1e-7, do_wstacking=True, flip_uw=False, out=None,
                   out_strides=None, accumulate=False, precision=None, slab=None):
    """One batch of a batched invert (sdp_hip_ms2dirty_batch): the batch is
    gridded into the resident w planes shared by the whole sequence; the
    ``first`` batch zeroes them, the ``last`` runs the FFT and w-screens into
    ``out`` (allocated if None; earlier batches return None).  ``bounds``:
    merge_bounds over every batch of the sequence.  ``slab`` = (lo, hi): grid
    only the visibilities whose first w plane of the sequence's layout
    (wstack_layout) lies in [lo, hi), into that slab's planes only
    (SDP_HIP_W_SLAB; the slabs of one layout sum to the full image)."""
    pbits = _prec_bits(epsilon, precision)
    _check_uvw(uvw)
    dev = uvw.device
    freq = _on_gpu(freq, "freq").to(torch.float64).contiguous()
    nrow, nchan = uvw.shape[0], freq.shape[0]
    if vis is not None:
        _on_gpu(vis, "vis")
        if vis.dtype not in (torch.complex64, torch.complex128) or tuple(vis.shape) != (nrow, nchan):
            raise ValueError("vis must be complex [nrow, nchan]")
    _check_wgt(wgt, nrow, nchan)
    if last:
        if out is None:
            # (never auto-release the workspace here: past the first batch it
            # holds the sequence's resident planes)
            out = _alloc((npix_x, npix_y), torch.float64, dev, may_release=first)
            out_strides = (npix_y, 1)
        elif out_strides is None:
            out_strides = out.stride()
        _on_gpu(out, "out")
        if out.dtype != torch.float64:
            raise ValueError("dirty output must be float64")
    if len(bounds) != 6:
        raise ValueError("bounds: {wmin, wmax, umax, vmax, fmin, fmax}")
    vals = [float(x) for x in bounds]
    if slab is not None:
        lo, hi = (int(x) for x in slab)
        if not 0 <= lo < hi:
            raise ValueError("slab: first planes (lo, hi) with 0 <= lo < hi")
        vals += [float(lo), float(hi)]
    bbuf = (ctypes.c_double * len(vals))(*vals)
    flags = ((_lib.SDP_HIP_FLIP_UW if flip_uw else 0) | (_lib.SDP_HIP_ACCUMULATE if accumulate else 0)
             | (_lib.SDP_HIP_BATCH_FIRST if first else 0) | (_lib.SDP_HIP_BATCH_LAST if last else 0)
             | (_lib.SDP_HIP_W_SLAB if slab is not None else 0) | pbits)
    info = _lib.WGridInfo()
    _lib.call(
        "sdp_hip_ms2dirty_batch",
        _ptr(uvw), uvw.stride(0), _ptr(freq), nchan, nrow,
        _ptr(vis), _DT_CODE[vis.dtype] if vis is not None else _lib.SDP_HIP_C64,
        vis.stride(0) if vis is not None else 0, vis.stride(1) if vis is not None else 0,
        *_wgt_args(wgt),
        int(npix_x), int(npix_y), float(pixsize_x), float(pixsize_y), float(epsilon),
        int(bool(do_wstacking)), flags, ctypes.cast(bbuf, ctypes.c_void_p),
        _ptr(out if last else None), int(out_strides[0]) if last else 0,
        int(out_strides[1]) if last else 0, _stream(dev), ctypes.byref(info))
    return (out if last else None), info.as_dict()


def _host3(v):
    """(l, m, n-1) as a host double[3] for the C ABI, or NULL."""
    if v is None:
        return None
    return ctypes.cast((ctypes.c_double * 3)(*[float(x) for x in v]), ctypes.c_void_p)


_FLAG_DT = {torch.int64: 8, torch.int32: 4, torch.int8: 1, torch.uint8: 1, torch.bool: 1}


def ms2dirty_vis(uvw, freq, vis, pol, wgt, flags, coef, npix_x, npix_y, pixsize_x, pixsize_y,
                 epsilon=1e-7, do_wstacking=True, flip_uw=False, out=None, out_strides=None,
                 accumulate=False, sumwt=None, shift_lmn=None, keep_buckets=False,
                 reuse_buckets=False, precision=None, slot=0, bounds=None, first=False,
                 last=False):
    """ms2dirty with invert_ng's visibility prologue fused in
    (sdp_hip_ms2dirty_vis): ``vis`` [nrow, nchan, npol_vis] complex (any
    strides, read in place; None = unit visibilities), ``flags`` the same
    shape (integer / bool, or None), ``wgt`` [nrow, nchan] f32/f64 weights of
    image pol ``pol``, ``coef`` the conversion-matrix row for that pol
    (complex [npol_vis]) or None for no conversion, ``sumwt`` a one-element
    f64 device view that receives += the masked weight sum.

    ``keep_buckets`` buckets every in-grid visibility and keeps the bucketing
    on the device; a following call with ``reuse_buckets`` and the same uvw,
    freq and geometry (another image pol) runs only the value pass, gridding
    and FFT (SDP_HIP_KEEP_BUCKETS / SDP_HIP_REUSE_BUCKETS).  ``slot=1`` uses
    the library's second scratch set (SDP_HIP_SLOT1; not with kept / reused
    buckets): calls alternated between two streams and slots overlap.

    ``bounds`` (uvw_bounds / merge_bounds of the whole sequence) makes the
    call one batch of a sequence sharing one set of resident w planes
    (sdp_hip_ms2dirty_vis_batch, as ms2dirty_batch): ``first`` zeroes them,
    ``last`` transforms them into ``out``."""
    pbits = _prec_bits(epsilon, precision)
    _check_uvw(uvw)
    dev = uvw.device
    freq = _on_gpu(freq, "freq").to(torch.float64).contiguous()
    nrow, nchan = uvw.shape[0], freq.shape[0]
    npv = 1
    if vis is not None:
        _on_gpu(vis, "vis")
        if vis.dtype not in (torch.complex64, torch.complex128) or vis.dim() != 3 or \
                tuple(vis.shape[:2]) != (nrow, nchan):
            raise ValueError("vis must be complex [nrow, nchan, npol]")
        npv = vis.shape[2]
    if flags is not None:
        _on_gpu(flags, "flags")
        if flags.dtype not in _FLAG_DT or flags.dim() != 3 or tuple(flags.shape[:2]) != (nrow, nchan):
            raise ValueError("flags must be an integer [nrow, nchan, npol] tensor")
        npv = max(npv, flags.shape[2])
    if wgt is not None:
        _on_gpu(wgt, "wgt")
        if wgt.dtype not in (torch.float32, torch.float64) or tuple(wgt.shape) != (nrow, nchan):
            raise ValueError("wgt must be float32/float64 [nrow, nchan]")
    if not 0 <= pol < npv:
        raise ValueError("pol out of range")
    cbuf = None
    if coef is not None:
        c = [complex(x) for x in coef]
        if len(c) != npv:
            raise ValueError("coef must have one entry per visibility pol")
        cbuf = (ctypes.c_double * (2 * npv))(*[v for z in c for v in (z.real, z.imag)])
    if out is None:
        out = _alloc((npix_x, npix_y), torch.float64, dev)
        out_strides = (npix_y, 1)
    elif out_strides is None:
        out_strides = out.stride()
    _on_gpu(out, "out")
    if out.dtype != torch.float64:
        raise ValueError("dirty output must be float64")
    if sumwt is not None and (sumwt.dtype != torch.float64 or not sumwt.is_cuda):
        raise ValueError("sumwt must be a float64 device tensor")
    bits = ((_lib.SDP_HIP_FLIP_UW if flip_uw else 0) | (_lib.SDP_HIP_ACCUMULATE if accumulate else 0)
            | pbits)
    bits |= (_lib.SDP_HIP_KEEP_BUCKETS if keep_buckets else 0) | \
        (_lib.SDP_HIP_REUSE_BUCKETS if reuse_buckets else 0) | (_lib.SDP_HIP_SLOT1 if slot else 0)
    info = _lib.WGridInfo()
    batch = ()
    name = "sdp_hip_ms2dirty_vis"
    if bounds is not None:
        if len(bounds) != 6:
            raise ValueError("bounds: {wmin, wmax, umax, vmax, fmin, fmax}")
        bits |= (_lib.SDP_HIP_BATCH_FIRST if first else 0) | (_lib.SDP_HIP_BATCH_LAST if last else 0)
        bbuf = (ctypes.c_double * 6)(*[float(x) for x in bounds])
        batch = (ctypes.cast(bbuf, ctypes.c_void_p),)
        name = "sdp_hip_ms2dirty_vis_batch"
    _lib.call(
        name,
        _ptr(uvw), uvw.stride(0), _ptr(freq), nchan, nrow,
        _ptr(vis), _DT_CODE[vis.dtype] if vis is not None else _lib.SDP_HIP_C64,
        *(vis.stride() if vis is not None else (0, 0, 0)), npv,
        ctypes.cast(cbuf, ctypes.c_void_p) if cbuf is not None else None,
        _ptr(wgt), _DT_CODE[wgt.dtype] if wgt is not None else _lib.SDP_HIP_F32,
        *(wgt.stride() if wgt is not None else (0, 0)),
        _ptr(flags), _FLAG_DT[flags.dtype] if flags is not None else 0,
        *(flags.stride() if flags is not None else (0, 0, 0)), int(pol),
        int(npix_x), int(npix_y), float(pixsize_x), float(pixsize_y), float(epsilon),
        int(bool(do_wstacking)), bits, *batch,
        _ptr(out), int(out_strides[0]), int(out_strides[1]), _ptr(sumwt), _host3(shift_lmn),
        _stream(dev), ctypes.byref(info))
    return out, info.as_dict()


def ms2dirty_vis_pols(uvw, freq, vis, wgt, flags, coef, npix_x, npix_y, pixsize_x, pixsize_y,
                      epsilon=1e-7, do_wstacking=True, flip_uw=False, out=None, out_strides=None,
                      accumulate=False, sumwt=None, shift_lmn=None, precision=None):
    """Every image pol of one invert_ng image channel in one call
    (sdp_hip_ms2dirty_vis_pols): ``vis`` [nrow, nchan, npol_vis] complex and
    ``flags`` (integer, or None) as ms2dirty_vis, ``wgt`` [nrow, nchan,
    >= npol_img] f32/f64 (image pol q takes the weights and flags of pol q),
    ``coef`` the conversion matrix [npol_img, npol_vis] (complex) or None for
    the identity.  ``out`` [npol_img, ...] f64 with ``out_strides`` = (pol,
    x, y) element strides; ``sumwt`` a [npol_img] f64 device view (+= each
    pol's masked weight sum).  The pols share one bucketing and one value
    pass; results as one ms2dirty_vis call per image pol."""
    pbits = _prec_bits(epsilon, precision)
    _check_uvw(uvw)
    dev = uvw.device
    freq = _on_gpu(freq, "freq").to(torch.float64).contiguous()
    nrow, nchan = uvw.shape[0], freq.shape[0]
    _on_gpu(vis, "vis")
    if vis.dtype not in (torch.complex64, torch.complex128) or vis.dim() != 3 or \
            tuple(vis.shape[:2]) != (nrow, nchan):
        raise ValueError("vis must be complex [nrow, nchan, npol]")
    npv = vis.shape[2]
    if flags is not None:
        _on_gpu(flags, "flags")
        if flags.dtype not in _FLAG_DT or tuple(flags.shape) != tuple(vis.shape):
            raise ValueError("flags must be an integer tensor shaped as vis")
    _on_gpu(wgt, "wgt")
    if wgt.dtype not in (torch.float32, torch.float64) or wgt.dim() != 3 or \
            tuple(wgt.shape[:2]) != (nrow, nchan):
        raise ValueError("wgt must be float32/float64 [nrow, nchan, npol]")
    npo = npv if coef is None else len(coef)
    if not 1 <= npo <= min(npv, wgt.shape[2]):
        raise ValueError("npol_img must be 1..npol_vis (and have weights)")
    cbuf = None
    if coef is not None:
        rows = [[complex(z) for z in r] for r in coef]
        if any(len(r) != npv for r in rows):
            raise ValueError("coef rows must have one entry per visibility pol")
        cbuf = (ctypes.c_double * (2 * npo * npv))(
            *[v for r in rows for z in r for v in (z.real, z.imag)])
    if out is None:
        out = _alloc((npo, npix_x, npix_y), torch.float64, dev)
        out_strides = out.stride()
    elif out_strides is None:
        out_strides = out.stride()
    _on_gpu(out, "out")
    if out.dtype != torch.float64:
        raise ValueError("dirty output must be float64")
    if sumwt is not None and (sumwt.dtype != torch.float64 or not sumwt.is_cuda or
                              sumwt.numel() < npo):
        raise ValueError("sumwt must be a float64 device tensor with one entry per image pol")
    bits = ((_lib.SDP_HIP_FLIP_UW if flip_uw else 0) | (_lib.SDP_HIP_ACCUMULATE if accumulate else 0)
            | pbits)
    info = _lib.WGridInfo()
    _lib.call(
        "sdp_hip_ms2dirty_vis_pols",
        _ptr(uvw), uvw.stride(0), _ptr(freq), nchan, nrow,
        _ptr(vis), _DT_CODE[vis.dtype], *vis.stride(), npv,
        ctypes.cast(cbuf, ctypes.c_void_p) if cbuf is not None else None, npo,
        _ptr(wgt), _DT_CODE[wgt.dtype], *wgt.stride(),
        _ptr(flags), _FLAG_DT[flags.dtype] if flags is not None else 0,
        *(flags.stride() if flags is not None else (0, 0, 0)),
        int(npix_x), int(npix_y), float(pixsize_x), float(pixsize_y), float(epsilon),
        int(bool(do_wstacking)), bits,
        _ptr(out), int(out_strides[1]), int(out_strides[2]), int(out_strides[0]),
        _ptr(sumwt), int(sumwt.stride(0)) if sumwt is not None else 0, _host3(shift_lmn),
        _stream(dev), ctypes.byref(info))
    return out, info.as_dict()


def dirty2ms_vis(uvw, freq, dirty, out, coef, pixsize_x, pixsize_y, epsilon=1e-7,
                 do_wstacking=True, flip_uw=False, dirty_strides=None, npix=None,
                 accumulate=False, shift_lmn=None, precision=None):
    """One image pol of predict_ng with the pol conversion fused into the
    write-back (sdp_hip_dirty2ms_vis): ``out`` [nrow, nchan, npol_vis] complex
    (any strides) gets coef[k] * predicted vis in pol k (coef None: pol 0)."""
    pbits = _prec_bits(epsilon, precision)
    _check_uvw(uvw)
    dev = uvw.device
    freq = _on_gpu(freq, "freq").to(torch.float64).contiguous()
    nrow, nchan = uvw.shape[0], freq.shape[0]
    _on_gpu(dirty, "dirty")
    if dirty.dtype != torch.float64:
        raise ValueError("dirty must be float64")
    npix_x, npix_y = (dirty.shape[-2], dirty.shape[-1]) if npix is None else npix
    if dirty_strides is None:
        dirty_strides = dirty.stride()[-2:]
    _on_gpu(out, "out")
    if out.dtype not in (torch.complex64, torch.complex128) or out.dim() != 3 or \
            tuple(out.shape[:2]) != (nrow, nchan):
        raise ValueError("out must be complex [nrow, nchan, npol]")
    npv = out.shape[2]
    cbuf = None
    if coef is not None:
        c = [complex(x) for x in coef]
        if len(c) != npv:
            raise ValueError("coef must have one entry per visibility pol")
        cbuf = (ctypes.c_double * (2 * npv))(*[v for z in c for v in (z.real, z.imag)])
    bits = ((_lib.SDP_HIP_FLIP_UW if flip_uw else 0) | (_lib.SDP_HIP_ACCUMULATE if accumulate else 0)
            | pbits)
    info = _lib.WGridInfo()
    _lib.call("sdp_hip_dirty2ms_vis", _ptr(uvw), uvw.stride(0), _ptr(freq), nchan, nrow,
              _ptr(dirty), int(dirty_strides[0]), int(dirty_strides[1]), int(npix_x), int(npix_y),
              float(pixsize_x), float(pixsize_y), float(epsilon), int(bool(do_wstacking)), bits,
              _ptr(out), _DT_CODE[out.dtype], *out.stride(), npv,
              ctypes.cast(cbuf, ctypes.c_void_p) if cbuf is not None else None,
              _host3(shift_lmn), _stream(dev), ctypes.byref(info))
    return out, info.as_dict()


def dirty2ms_vis_pols(uvw, freq, dirty, out, coef, pixsize_x, pixsize_y, epsilon=1e-7,
                      do_wstacking=True, flip_uw=False, dirty_strides=None, npix=None,
                      accumulate=False, shift_lmn=None, precision=None):
    """Every image pol of predict_ng in one call (sdp_hip_dirty2ms_vis_pols):
    ``dirty`` [npol_img, ...] f64 with ``dirty_strides`` = (pol, x, y),
    ``out`` [nrow, nchan, npol_vis] complex (any strides) gets
    sum_q coef[q][k] * prediction_q in vis pol k (coef None: identity).  The
    pols share one bucketing and one write-back; results as one dirty2ms_vis
    call per image pol, accumulating after the first."""
    pbits = _prec_bits(epsilon, precision)
    _check_uvw(uvw)
    dev = uvw.device
    freq = _on_gpu(freq, "freq").to(torch.float64).contiguous()
    nrow, nchan = uvw.shape[0], freq.shape[0]
    _on_gpu(dirty, "dirty")
    if dirty.dtype != torch.float64 or dirty.dim() != 3:
        raise ValueError("dirty must be float64 [npol_img, nx, ny]")
    npo = dirty.shape[0]
    npix_x, npix_y = (dirty.shape[-2], dirty.shape[-1]) if npix is None else npix
    if dirty_strides is None:
        dirty_strides = dirty.stride()
    _on_gpu(out, "out")
    if out.dtype not in (torch.complex64, torch.complex128) or out.dim() != 3 or \
            tuple(out.shape[:2]) != (nrow, nchan):
        raise ValueError("out must be complex [nrow, nchan, npol]")
    npv = out.shape[2]
    if not 1 <= npo <= 4:
        raise ValueError("npol_img must be 1..4")
    cbuf = None
    if coef is not None:
        rows = [[complex(z) for z in r] for r in coef]
        if len(rows) != npo or any(len(r) != npv for r in rows):
            raise ValueError("coef must be [npol_img][npol_vis]")
        cbuf = (ctypes.c_double * (2 * npo * npv))(
            *[v for r in rows for z in r for v in (z.real, z.imag)])
    bits = ((_lib.SDP_HIP_FLIP_UW if flip_uw else 0) | (_lib.SDP_HIP_ACCUMULATE if accumulate else 0)
            | pbits)
    info = _lib.WGridInfo()
    _lib.call("sdp_hip_dirty2ms_vis_pols", _ptr(uvw), uvw.stride(0), _ptr(freq), nchan, nrow,
              _ptr(dirty), int(dirty_strides[1]), int(dirty_strides[2]), int(dirty_strides[0]),
              npo, int(npix_x), int(npix_y), float(pixsize_x), float(pixsize_y), float(epsilon),
              int(bool(do_wstacking)), bits, _ptr(out), _DT_CODE[out.dtype], *out.stride(), npv,
              ctypes.cast(cbuf, ctypes.c_void_p) if cbuf is not None else None,
              _host3(shift_lmn), _stream(dev), ctypes.byref(info))
    return out, info.as_dict()


def dirty2ms(uvw, freq, dirty, wgt, pixsize_x, pixsize_y, epsilon=1e-7,
             do_wstacking=True, flip_uw=False, out=None, dirty_strides=None,
             npix=None, accumulate=False, vis_dtype=torch.complex64, precision=None):
    """ducc0.wgridder.dirty2ms semantics on device; returns vis [nrow,nchan]."""
    pbits = _prec_bits(epsilon, precision)
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
    _check_wgt(wgt, nrow, nchan)
    if out is None:
        out = _alloc((nrow, nchan), vis_dtype, dev)
    _on_gpu(out, "vis out")
    if out.dtype not in (torch.complex64, torch.complex128) or tuple(out.shape) != (nrow, nchan):
        raise ValueError("vis out must be complex [nrow, nchan]")
    flags = ((_lib.SDP_HIP_FLIP_UW if flip_uw else 0) | (_lib.SDP_HIP_ACCUMULATE if accumulate else 0)
             | pbits)
    info = _lib.WGridInfo()
    _lib.call(
        "sdp_hip_dirty2ms",
        _ptr(uvw), uvw.stride(0), _ptr(freq), nchan, nrow,
        _ptr(dirty), int(dirty_strides[0]), int(dirty_strides[1]), int(npix_x), int(npix_y),
        float(pixsize_x), float(pixsize_y),
        *_wgt_args(wgt),
        float(epsilon), int(bool(do_wstacking)), flags,
        _ptr(out), _DT_CODE[out.dtype], out.stride(0), out.stride(1),
        _stream(dev), ctypes.byref(info))
    return out, info.as_dict()


def set_stage_timing(enable):
    _lib.load().sdp_hip_set_stage_timing(int(bool(enable)))


def release_workspace():
    _lib.call("sdp_hip_release_workspace")


def dft_point(direction_cosines, fluxes, uvw, freq=None, out=None, vis_dtype=torch.complex64):
    """Sky-component DFT on device.

    direction_cosines [ncomp,3] f64, fluxes [ncomp, 1|nchan, npol] c128.
    With ``freq`` given, ``uvw`` is [nrow,3] metres (lambda scaling fused);
    otherwise ``uvw`` is uvw_lambda [nrow, nchan, 3] (dft_point_v00 layout).
    Returns vis [nrow, nchan, npol].
    """
    dc = _on_gpu(direction_cosines, "direction_cosines").to(torch.float64).contiguous()
    fl = _on_gpu(fluxes, "fluxes").to(torch.complex128).contiguous()
    if fl.dim() != 3 or dc.dim() != 2 or dc.shape[1] != 3 or fl.shape[0] != dc.shape[0]:
        raise ValueError("direction_cosines [ncomp,3] and fluxes [ncomp,nchan,npol] required")
    ncomp, fnchan, npol = fl.shape
    uvw = _on_gpu(uvw, "uvw").to(torch.float64).contiguous()
    if freq is not None:
        freq = _on_gpu(freq, "freq").to(torch.float64).contiguous()
        nrow, nchan = uvw.shape[0], freq.shape[0]
    else:
        nrow, nchan = uvw.shape[0], uvw.shape[1]
    if out is None:
        out = _alloc((nrow, nchan, npol), vis_dtype, uvw.device)
    if not out.is_contiguous() or tuple(out.shape) != (nrow, nchan, npol):
        raise ValueError("vis out must be contiguous [nrow, nchan, npol]")
    if freq is not None:
        _lib.call("sdp_hip_dft_point_metres", ncomp, _ptr(dc), _ptr(fl), fnchan, npol, nrow, nchan,
                  _ptr(uvw), _ptr(freq), _ptr(out), _DT_CODE[out.dtype], _stream(uvw.device))
    else:
        _lib.call("sdp_hip_dft_point_v00", ncomp, _ptr(dc), _ptr(fl), fnchan, npol, nrow, nchan,
                  _ptr(uvw), _ptr(out), _DT_CODE[out.dtype], _stream(uvw.device))
    return out


def canonical_baselines(ant1, ant2, nants):
    """Canonical (a1 < a2) CSR order of a baseline list.

    Returns (perm, conj, row_start, ant2_sorted): ``perm[k]`` is the input
    baseline placed at canonical position k, ``conj[k]`` is True when it was
    given as (a2, a1) (its value must be conjugated), and autocorrelations
    (a1 == a2, zeroed by the reference solver, solvers.py:251-253) are dropped.
    """
    import numpy as np
    a1 = np.asarray(ant1, dtype=np.int64)
    a2 = np.asarray(ant2, dtype=np.int64)
    keep = np.nonzero(a1 != a2)[0]
    lo = np.minimum(a1[keep], a2[keep])
    hi = np.maximum(a1[keep], a2[keep])
    order = np.lexsort((hi, lo))
    perm = keep[order]
    conj = (a1[perm] > a2[perm])
    lo, hi = lo[order], hi[order]
    row_start = np.zeros(nants + 1, dtype=np.int32)
    np.add.at(row_start, lo + 1, 1)
    row_start = np.cumsum(row_start).astype(np.int32)
    return perm, conj, row_start, hi.astype(np.int32)


def solve_gains(xb, wb, gain, gwt, row_start, ant2, mode, niter=200, tol=1e-6,
                phase_only=True, refant=0, damping=0.5):
    """Batched StefCal on device.

    xb [nsolve, nbl, nchan, npol] c128, wb [...] f64 in canonical baseline
    order; gain/gwt [nsolve, nants, nchan, nrec, nrec] (c128 / f64) updated
    in place.  Returns (residual [nsolve, nchan, nrec, nrec], niter_used).
    """
    xb = _on_gpu(xb, "xb").to(torch.complex128).contiguous()
    wb = _on_gpu(wb, "wb").to(torch.float64).contiguous()
    if not (gain.is_cuda and gain.dtype == torch.complex128 and gain.is_contiguous()):
        raise ValueError("gain must be a contiguous complex128 device tensor")
    if not (gwt.is_cuda and gwt.dtype == torch.float64 and gwt.is_contiguous()):
        raise ValueError("gwt must be a contiguous float64 device tensor")
    nsolve, nbl, nchan, npol = xb.shape
    nants = gain.shape[1]
    nrec = gain.shape[3]
    rs = torch.as_tensor(row_start, dtype=torch.int32, device=xb.device)
    a2 = torch.as_tensor(ant2, dtype=torch.int32, device=xb.device)
    residual = torch.zeros((nsolve, nchan, nrec, nrec), dtype=torch.float64, device=xb.device)
    used = torch.zeros(nsolve, dtype=torch.int32, device=xb.device)
    _lib.call("sdp_hip_solve_gains", nsolve, nants, nbl, _ptr(rs), _ptr(a2), nchan, npol,
              int(mode), _ptr(xb), _ptr(wb), _ptr(gain), _ptr(gwt), _ptr(residual), _ptr(used),
              int(niter), float(tol), int(bool(phase_only)), int(refant), float(damping),
              _stream(xb.device))
    return residual, used


def _check_cf_operands(maps, vis_to_im, cf, grid, nrow, nchan, npol):
    """Operand checks shared by grid_cf / degrid_cf: dtypes, contiguity,
    shapes, and the image channel of every visibility channel.  The
    reference indexes ``gd[imchan]`` / ``cf[imchan]`` with numpy
    (grid_data/gridding.py:226-245, :560-580): an index past the GridData's
    (or the CF's) channel axis raises IndexError and a negative one counts
    from the end, so vis_to_im is checked here and negatives are wrapped.
    Returns the (possibly wrapped) int32 vis_to_im on the device."""
    cfn, cf_npol, _, _, _, gv, gu = cf.shape
    gn, g_npol, ny, nx = grid.shape
    if cf.dtype != torch.complex128 or grid.dtype != torch.complex128:
        raise ValueError("cf and grid must be complex128")
    if not (cf.is_contiguous() and grid.is_contiguous()):
        raise ValueError("cf and grid must be contiguous")
    if cf_npol != npol or g_npol != npol:
        raise ValueError(f"pol axes differ: vis {npol}, cf {cf_npol}, grid {g_npol}")
    for k in ("pu", "pv", "pwc", "pdu", "pdv"):
        m = maps[k]
        if m.dtype != torch.int32 or not m.is_contiguous() or tuple(m.shape) != (nchan, nrow):
            raise ValueError(f"map {k} must be contiguous int32 [{nchan}, {nrow}]")
    v2i = vis_to_im.detach().to("cpu", torch.int64)
    if v2i.numel() != nchan:
        raise ValueError(f"vis_to_im has {v2i.numel()} entries for {nchan} channels")
    lim = min(gn, cfn)
    if bool((v2i >= lim).any()) or bool((v2i < -lim).any()):
        raise IndexError(f"vis_to_im {v2i.tolist()} out of range for {gn} grid / {cfn} cf "
                         "channels")
    if bool((v2i < 0).any()):
        # numpy wraps gd[imchan] by the grid's channel count and cf[imchan] by
        # the CF's: one kernel index serves both only when the counts agree
        if gn != cfn:
            raise IndexError(f"negative vis_to_im {v2i.tolist()} with {gn} grid and {cfn} cf "
                             "channels: the reference would pick different grid and cf "
                             "channels; pass non-negative channel indices")
        v2i = torch.where(v2i < 0, v2i + gn, v2i)
    return v2i.to(device=grid.device, dtype=torch.int32)


def grid_cf(maps, vis_to_im, vis, wt, cf, grid, sumwt):
    """Convolution-function gridding (accumulates into grid and sumwt).

    maps: dict of int32 [nchan, nrow] device tensors pu, pv, pwc, pdu, pdv;
    vis [nrow, nchan, npol] c128, wt f64 same shape; cf [c, p, nw, ndv, ndu,
    gv, gu] c128; grid [g_nchan, npol, ny, nx] c128; sumwt [g_nchan, npol] f64.
    Returns the number of skipped (row, pol) samples.
    """
    nrow, nchan, npol = vis.shape
    cfn, _, nw, ndv, ndu, gv, gu = cf.shape
    gn, _, ny, nx = grid.shape
    if vis.dtype != torch.complex128 or wt.dtype != torch.float64 or sumwt.dtype != torch.float64:
        raise ValueError("grid_cf: vis complex128, wt and sumwt float64")
    if tuple(wt.shape) != (nrow, nchan, npol) or tuple(sumwt.shape) != (gn, npol):
        raise ValueError("grid_cf: wt must match vis, sumwt must be [g_nchan, npol]")
    for t in (vis, wt, sumwt):
        if not t.is_contiguous():
            raise ValueError("grid_cf operands must be contiguous")
    v2i = _check_cf_operands(maps, vis_to_im, cf, grid, nrow, nchan, npol)
    skipped = torch.zeros(1, dtype=torch.int64, device=vis.device)
    _lib.call("sdp_hip_grid_cf", nrow, nchan, npol, _ptr(maps["pu"]), _ptr(maps["pv"]),
              _ptr(maps["pwc"]), _ptr(maps["pdu"]), _ptr(maps["pdv"]), _ptr(v2i), _ptr(vis),
              _ptr(wt), _ptr(cf), cfn, nw, ndv, ndu, gv, gu, _ptr(grid), gn, ny, nx, _ptr(sumwt),
              _ptr(skipped), _stream(vis.device))
    return skipped


def degrid_cf(maps, vis_to_im, grid, cf, nrow, nchan, out):
    """Convolution-function degridding into out [nrow, nchan, npol] c128
    (skipped samples are written as zero).  Returns the skipped count."""
    cfn, npol, nw, ndv, ndu, gv, gu = cf.shape
    gn, _, ny, nx = grid.shape
    if out.dtype != torch.complex128 or not out.is_contiguous() or \
            tuple(out.shape) != (nrow, nchan, npol):
        raise ValueError(f"degrid_cf: out must be contiguous complex128 [{nrow}, {nchan}, {npol}]")
    v2i = _check_cf_operands(maps, vis_to_im, cf, grid, nrow, nchan, npol)
    skipped = torch.zeros(1, dtype=torch.int64, device=grid.device)
    _lib.call("sdp_hip_degrid_cf", nrow, nchan, npol, _ptr(maps["pu"]), _ptr(maps["pv"]),
              _ptr(maps["pwc"]), _ptr(maps["pdu"]), _ptr(maps["pdv"]), _ptr(v2i),
              _ptr(grid), gn, ny, nx, _ptr(cf), cfn, nw, ndv, ndu, gv, gu, _ptr(out),
              _ptr(skipped), _stream(grid.device))
    return skipped


# ---- imaging weights (sdp_hip_grid_weights / sdp_hip_reweight / sdp_hip_taper)
_FLAG_BYTES = {torch.int64: 8, torch.int32: 4, torch.int8: 1, torch.uint8: 1, torch.bool: 1}
WEIGHTING = {"natural": 0, "uniform": 1, "robust": 2}


def _weight_operands(uvw, freq, weight, flags):
    _check_uvw(uvw)
    for t, n in ((freq, "freq"), (weight, "weight")):
        _on_gpu(t, n)
        if t.dtype != torch.float64 or not t.is_contiguous():
            raise ValueError(f"{n} must be a contiguous float64 device tensor")
    if not uvw.is_contiguous():
        raise ValueError("uvw must be contiguous [nrow, 3]")
    nrow, nchan, npol = weight.shape
    if uvw.shape[0] != nrow or freq.numel() != nchan:
        raise ValueError("weight must be [nrow, nchan, npol] matching uvw and freq")
    fb = 0
    if flags is not None:
        _on_gpu(flags, "flags")
        if flags.shape != weight.shape or not flags.is_contiguous() or flags.dtype not in _FLAG_BYTES:
            raise ValueError("flags must be a contiguous integer tensor shaped like weight")
        fb = _FLAG_BYTES[flags.dtype]
    return nrow, nchan, npol, fb


def _wcs6(wcs):
    return torch.tensor([float(x) for ax in wcs for x in ax], dtype=torch.float64)


def grid_weights(uvw, freq, weight, flags, vis_to_im, wcs, grid, sumwt):
    """Accumulate flagged weights into ``grid`` [g_nchan, npol, ny, nx] f64 and
    ``sumwt`` [g_nchan, npol]; ``wcs`` = ((crval, cdelt, crpix) of UU, of VV).
    Returns the device count of skipped (row, chan, pol) samples."""
    nrow, nchan, npol, fb = _weight_operands(uvw, freq, weight, flags)
    gn, gp, ny, nx = grid.shape
    if gp != npol or grid.dtype != torch.float64 or not grid.is_contiguous():
        raise ValueError("grid must be contiguous float64 [g_nchan, npol, ny, nx]")
    if sumwt.shape != (gn, npol) or sumwt.dtype != torch.float64:
        raise ValueError("sumwt must be float64 [g_nchan, npol]")
    w6 = _wcs6(wcs).to(uvw.device)
    skipped = torch.zeros(1, dtype=torch.int64, device=uvw.device)
    _lib.call("sdp_hip_grid_weights", nrow, nchan, npol, _ptr(uvw), _ptr(freq), _ptr(weight),
              _ptr(flags), fb, _ptr(vis_to_im), _ptr(w6), _ptr(grid), gn, ny, nx, _ptr(sumwt),
              _ptr(skipped), _stream(uvw.device))
    return skipped


def reweight(uvw, freq, weight, flags, vis_to_im, wcs, grid, imaging_weight, weighting="uniform",
             robustness=0.0, sumwt=None):
    """Overwrite ``imaging_weight`` [nrow, nchan, npol] f64 in place."""
    if weighting not in WEIGHTING:
        raise AssertionError(f"Weighting {weighting} not supported")
    nrow, nchan, npol, fb = _weight_operands(uvw, freq, weight, flags)
    _on_gpu(imaging_weight, "imaging_weight")
    if (imaging_weight.shape != weight.shape or imaging_weight.dtype != torch.float64
            or not imaging_weight.is_contiguous()):
        raise ValueError("imaging_weight must be contiguous float64 shaped like weight")
    coef = (5.0 * 10.0 ** (-robustness)) ** 2
    if grid is None:
        gn, ny, nx, w6 = 1, 1, 1, torch.tensor([0.0, 1.0, 1.0, 0.0, 1.0, 1.0], dtype=torch.float64)
    else:
        gn, _, ny, nx = grid.shape
        w6 = _wcs6(wcs)
    w6 = w6.to(uvw.device)
    ns = 0 if sumwt is None else sumwt.numel()
    _lib.call("sdp_hip_reweight", nrow, nchan, npol, _ptr(uvw), _ptr(freq), _ptr(weight),
              _ptr(flags), fb, _ptr(vis_to_im), _ptr(w6), _ptr(grid), gn, ny, nx,
              WEIGHTING[weighting], coef, _ptr(sumwt), ns, _ptr(imaging_weight),
              _stream(uvw.device))
    return imaging_weight


def taper(uvw, freq, flags, imaging_weight, kind, param):
    """In place: imaging_weight = flagged imaging weight * taper; kind
    "gaussian" (param = pi^2 beam^2 / (4 ln 2)) or "tukey" (param = r)."""
    nrow, nchan, npol, fb = _weight_operands(uvw, freq, imaging_weight, flags)
    _lib.call("sdp_hip_taper", nrow, nchan, npol, _ptr(uvw), _ptr(freq), _ptr(flags), fb,
              {"gaussian": 0, "tukey": 1}[kind], float(param), _ptr(imaging_weight),
              _stream(uvw.device))
    return imaging_weight


# ---- calibration neighbours (sdp_hip_point_sums / divide_vis / apply_gains)
def _vis4(t, name):
    _on_gpu(t, name)
    if t.dtype not in (torch.complex64, torch.complex128) or t.dim() != 4 or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous complex [t, b, f, p] tensor")
    return t


def _flags_of(flags, shape):
    if flags is None:
        return None, 0
    _on_gpu(flags, "flags")
    if tuple(flags.shape) != tuple(shape) or not flags.is_contiguous() or flags.dtype not in _FLAG_DT:
        raise ValueError("flags must be a contiguous integer tensor shaped like vis")
    return flags, _FLAG_DT[flags.dtype]


def point_sums(vis, model, weight, flags, row_ptr, time_idx, nchan_g, perm=None, conj=None,
               model_flags=None):
    """x_b, xwt_b [nrow_g, nbl, nchan_g, npol] (c128, f64) of solve_gaintable
    over divide_visibility(vis, model) (model None: vis itself)."""
    _vis4(vis, "vis")
    if model is not None:
        _vis4(model, "model")
        if model.shape != vis.shape or model.dtype != vis.dtype:
            raise ValueError("model must match vis")
    nt, nbl, nchan, npol = vis.shape
    if weight is not None and (weight.shape != vis.shape or weight.dtype != torch.float64
                               or not weight.is_contiguous()):
        raise ValueError("weight must be contiguous float64 shaped like vis")
    fl, fb = _flags_of(flags, vis.shape)
    nrow_g = row_ptr.numel() - 1
    nout = nbl if perm is None else perm.numel()
    if perm is not None and (perm.dtype != torch.int32 or (conj is not None and (
            conj.dtype != torch.uint8 or conj.numel() != nout))):
        raise ValueError("perm must be int32 and conj uint8 of the same length")
    xb = torch.empty((nrow_g, nout, nchan_g, npol), dtype=torch.complex128, device=vis.device)
    xwt = torch.empty((nrow_g, nout, nchan_g, npol), dtype=torch.float64, device=vis.device)
    mfl = _model_flags(model_flags, fl)
    _lib.call("sdp_hip_point_sums", nt, nbl, nchan, npol, _ptr(vis), _ptr(model),
              _DT_CODE[vis.dtype], _ptr(weight), _ptr(fl), _ptr(mfl), fb, nrow_g, _ptr(row_ptr),
              _ptr(time_idx), int(nchan_g), int(nout), _ptr(perm), _ptr(conj), _ptr(xb),
              _ptr(xwt), _stream(vis.device))
    return xb, xwt


def _model_flags(model_flags, fl):
    """The model's own flags in the vis flags' dtype, or None."""
    if model_flags is None or fl is None:
        return None
    _on_gpu(model_flags, "model_flags")
    if model_flags.shape != fl.shape:
        raise ValueError("model flags must be shaped like vis")
    return model_flags.to(fl.dtype).contiguous()


def divide_vis(vis, model, weight, flags, model_flags=None):
    """(x, xwt) of divide_visibility, same shapes as vis."""
    _vis4(vis, "vis")
    _vis4(model, "model")
    if model.shape != vis.shape or model.dtype != vis.dtype:
        raise ValueError("model must match vis")
    fl, fb = _flags_of(flags, vis.shape)
    x = torch.empty_like(vis)
    xwt = torch.empty(vis.shape, dtype=torch.float64, device=vis.device)
    mfl = _model_flags(model_flags, fl)
    _lib.call("sdp_hip_divide_vis", vis.numel(), _ptr(vis), _ptr(model), _DT_CODE[vis.dtype],
              _ptr(weight), _ptr(fl), _ptr(mfl), fb, _ptr(x), _ptr(xwt), _stream(vis.device))
    return x, xwt


def apply_gains(vis, weight, flags, use_flags, ant1, ant2, time_row, gain, inverse):
    """apply_gaintable in place on device vis / weight [t, b, f, p]."""
    _vis4(vis, "vis")
    nt, nbl, nchan, npol = vis.shape
    if weight.shape != vis.shape or weight.dtype != torch.float64 or not weight.is_contiguous():
        raise ValueError("weight must be contiguous float64 shaped like vis")
    fl, fb = _flags_of(flags, vis.shape)
    _on_gpu(gain, "gain")
    if gain.dtype != torch.complex128 or gain.dim() != 5 or not gain.is_contiguous():
        raise ValueError("gain must be contiguous complex128 [rows, nants, nchan, nrec, nrec]")
    nrow_g, nants, nchan_g, nrec, _ = gain.shape
    _lib.call("sdp_hip_apply_gains", nt, nbl, nchan, npol, _ptr(vis), _DT_CODE[vis.dtype],
              _ptr(weight), _ptr(fl), fb, int(bool(use_flags)), _ptr(ant1), _ptr(ant2),
              _ptr(time_row), _ptr(gain), nrow_g, nants, nchan_g, nrec, int(bool(inverse)),
              _stream(vis.device))
    return vis, weight
