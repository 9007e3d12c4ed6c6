"""Minimal ska-sdp-datamodels-compatible containers.

ska-sdp-datamodels 0.2.1 (with xarray and astropy) is the reference's data
layer but is not installed here; this module provides just the attribute
surface the hot path touches:

* ``Visibility`` ``[time, baseline, chan, pol]`` with ``vis``, ``uvw``,
  ``weight``, ``imaging_weight``, ``flags``, ``frequency``, ``baselines`` ...
  and ``visibility_acc`` (``flagged_vis``, ``uvw_lambda``, ...).
* ``Image`` ``[chan, pol, y, x]`` with a linear ``RA---SIN/DEC--SIN/STOKES/FREQ``
  WCS subset (``cdelt``, ``crpix``, ``crval``, ``sub``, ``wcs_world2pix``).
* ``GainTable``, ``SkyComponent``, ``GridData``, ``ConvolutionFunction``,
  ``PolarisationFrame`` and ``convert_pol_frame``.

Data variables may hold numpy arrays (host) or torch tensors on the GPU
(device-resident data for the benchmark path); the compute entry points
accept both.  If the real datamodels objects are passed, the hot-path
functions only use attributes that exist on both.
"""

import copy as _copy
import math

import numpy as np

try:  # torch is optional for the host-only containers
    import torch
except ImportError:  # pragma: no cover
    torch = None

C_M_S = 299792458.0


# ---------------------------------------------------------------------------
# sky coordinates (ICRS, radians) -- replaces astropy.SkyCoord on the hot path
# ---------------------------------------------------------------------------
class _Angle:
    def __init__(self, rad):
        self.rad = float(rad)

    @property
    def deg(self):
        return math.degrees(self.rad)


class SkyCoord:
    """ICRS direction in radians with the attributes the hot path uses."""

    def __init__(self, ra, dec, unit="rad", frame="icrs", equinox="J2000"):
        if unit == "deg":
            ra, dec = math.radians(ra), math.radians(dec)
        self.ra = _Angle(ra)
        self.dec = _Angle(dec)
        self.frame = frame
        self.equinox = equinox

    def separation(self, other):
        """Great-circle separation (haversine, stable at small angles)."""
        d_ra = other.ra.rad - self.ra.rad
        s = math.sin(0.5 * (other.dec.rad - self.dec.rad)) ** 2 + math.cos(self.dec.rad) * math.cos(
            other.dec.rad) * math.sin(0.5 * d_ra) ** 2
        return _Angle(2.0 * math.asin(min(1.0, math.sqrt(s))))

    def __eq__(self, other):
        return isinstance(other, SkyCoord) and self.ra.rad == other.ra.rad and self.dec.rad == other.dec.rad

    def __repr__(self):
        return f"SkyCoord(ra={self.ra.deg:.6f}deg, dec={self.dec.deg:.6f}deg)"


# ---------------------------------------------------------------------------
# polarisation frames
# ---------------------------------------------------------------------------
class PolarisationFrame:
    fpol_names = {
        "circular": ["RR", "RL", "LR", "LL"],
        "circularnp": ["RR", "LL"],
        "linear": ["XX", "XY", "YX", "YY"],
        "linearnp": ["XX", "YY"],
        "stokesIQUV": ["I", "Q", "U", "V"],
        "stokesIV": ["I", "V"],
        "stokesIQ": ["I", "Q"],
        "stokesI": ["I"],
    }

    def __init__(self, name):
        if name not in self.fpol_names:
            raise ValueError(f"Unknown polarisation frame {name}")
        self.type = name
        self.translations = {p: i for i, p in enumerate(self.fpol_names[name])}

    @property
    def npol(self):
        return len(self.fpol_names[self.type])

    @property
    def names(self):
        return list(self.fpol_names[self.type])

    def __eq__(self, other):
        if isinstance(other, str):
            return self.type == other
        return isinstance(other, PolarisationFrame) and self.type == other.type

    def __hash__(self):
        return hash(self.type)

    def __repr__(self):
        return f"PolarisationFrame('{self.type}')"


# Conversion matrices (rows: output pols, columns: input pols) following the
# ska-sdp-datamodels / RASCIL conventions: XX = I+Q, XY = U+iV, YX = U-iV,
# YY = I-Q; RR = I+V, RL = U-iQ, LR = U+iQ, LL = I-V.
_S2L = np.array([[1, 1, 0, 0], [0, 0, 1, 1j], [0, 0, 1, -1j], [1, -1, 0, 0]], dtype=complex)
_S2C = np.array([[1, 0, 0, 1], [0, -1j, 1, 0], [0, 1j, 1, 0], [1, 0, 0, -1]], dtype=complex)
_SQ2LNP = np.array([[1, 1], [1, -1]], dtype=complex)
_SV2CNP = np.array([[1, 1], [1, -1]], dtype=complex)

_CONVERSIONS = {
    ("stokesIQUV", "linear"): _S2L,
    ("linear", "stokesIQUV"): np.linalg.inv(_S2L),
    ("stokesIQUV", "circular"): _S2C,
    ("circular", "stokesIQUV"): np.linalg.inv(_S2C),
    ("stokesIQ", "linearnp"): _SQ2LNP,
    ("linearnp", "stokesIQ"): np.linalg.inv(_SQ2LNP),
    ("stokesIV", "circularnp"): _SV2CNP,
    ("circularnp", "stokesIV"): np.linalg.inv(_SV2CNP),
}


def pol_conversion_matrix(ipf, opf):
    """Matrix M with out[..., o] = sum_i M[o, i] in[..., i] (None = identity)."""
    if ipf == opf:
        return None
    key = (ipf.type, opf.type)
    if key not in _CONVERSIONS:
        raise ValueError(f"Unknown polarisation conversion: {ipf} to {opf}")
    return _CONVERSIONS[key]


def convert_pol_frame(polvec, ipf, opf, polaxis=1):
    """Convert polarisation frame along ``polaxis`` (numpy or torch)."""
    m = pol_conversion_matrix(ipf, opf)
    if m is None:
        return polvec
    if torch is not None and isinstance(polvec, torch.Tensor):
        mt = torch.as_tensor(m, device=polvec.device,
                             dtype=polvec.dtype if polvec.is_complex() else torch.complex128)
        x = torch.movedim(polvec.to(mt.dtype), polaxis, -1)
        return torch.movedim(x @ mt.T, -1, polaxis)
    x = np.moveaxis(np.asarray(polvec), polaxis, -1)
    return np.moveaxis(x @ m.T, -1, polaxis)


# ---------------------------------------------------------------------------
# a small xarray stand-in
# ---------------------------------------------------------------------------
def _clone(a, zero=False):
    if torch is not None and isinstance(a, torch.Tensor):
        return torch.zeros_like(a) if zero else a.clone()
    a = np.asarray(a)
    return np.zeros_like(a) if zero else a.copy()


class DataArray:
    def __init__(self, owner, name):
        object.__setattr__(self, "_owner", owner)
        object.__setattr__(self, "_name", name)

    @property
    def data(self):
        return self._owner._vars[self._name]

    @data.setter
    def data(self, value):
        self._owner._vars[self._name] = value

    @property
    def values(self):
        d = self.data
        return d.cpu().numpy() if torch is not None and isinstance(d, torch.Tensor) else d

    @property
    def shape(self):
        return tuple(self.data.shape)

    @property
    def dtype(self):
        return self.data.dtype

    def __getitem__(self, key):
        return self.data[key]

    def __setitem__(self, key, value):
        self.data[key] = value

    def __array__(self, dtype=None, copy=None):
        v = np.asarray(self.values)
        return v.astype(dtype) if dtype is not None else v

    def __len__(self):
        return len(self.data)

    def __iter__(self):
        return iter(self.data)

    def sum(self, *a, **k):
        return self.data.sum(*a, **k)


class _Derived(DataArray):
    """Read-only DataArray over a computed value (``visibility_acc.u`` etc.,
    which the reference reads through ``.data``, weighting.py:93)."""

    def __init__(self, value):
        object.__setattr__(self, "_value", value)

    @property
    def data(self):
        return self._value


class Dataset:
    """Variables live in ``_vars``; ``ds[name].data`` and ``ds.name`` both work."""

    _var_names = ()

    def __init__(self, variables, attrs=None):
        object.__setattr__(self, "_vars", dict(variables))
        object.__setattr__(self, "attrs", dict(attrs or {}))

    def __getitem__(self, name):
        if name not in self._vars:
            raise KeyError(name)
        return DataArray(self, name)

    def __setitem__(self, name, value):
        self._vars[name] = value.data if isinstance(value, DataArray) else value

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        if name in self._vars:
            return DataArray(self, name)
        if name in self.attrs:
            return self.attrs[name]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in self._vars:
            self._vars[name] = value.data if isinstance(value, DataArray) else value
        else:
            object.__setattr__(self, name, value)

    def _copy_with(self, deep=True, zero_vars=(), replace=None):
        new = object.__new__(type(self))
        variables = {}
        replace = replace or {}
        for k, v in self._vars.items():
            if k in replace:
                variables[k] = replace[k]
            elif deep:
                variables[k] = _clone(v, zero=k in zero_vars)
            else:
                variables[k] = v
        object.__setattr__(new, "_vars", variables)
        object.__setattr__(new, "attrs", _copy.deepcopy(self.attrs) if deep else dict(self.attrs))
        return new


# ---------------------------------------------------------------------------
# WCS subset
# ---------------------------------------------------------------------------
class _WcsParams:
    def __init__(self, ctype, crpix, cdelt, crval, cunit=None):
        self.ctype = list(ctype)
        self.crpix = np.array(crpix, dtype=float)
        self.cdelt = np.array(cdelt, dtype=float)
        self.crval = np.array(crval, dtype=float)
        self.cunit = list(cunit) if cunit is not None else [""] * len(ctype)
        self.radesys = "ICRS"
        self.equinox = 2000.0


class WCS:
    """Linear WCS: world = crval + cdelt * (pix + 1 - crpix) (origin 0).

    Celestial axes are only used through their cdelt/crval/crpix (the hot path
    deprojects SIN itself, see ``pixel_to_skycoord``)."""

    def __init__(self, naxis=4, ctype=None, crpix=None, cdelt=None, crval=None, cunit=None):
        ctype = ctype or [""] * naxis
        self.wcs = _WcsParams(ctype, crpix or [0.0] * naxis, cdelt or [1.0] * naxis,
                              crval or [0.0] * naxis, cunit)
        self.naxis = naxis

    def sub(self, axes):
        idx = [a - 1 for a in axes]
        w = WCS(len(idx), [self.wcs.ctype[i] for i in idx], [self.wcs.crpix[i] for i in idx],
                [self.wcs.cdelt[i] for i in idx], [self.wcs.crval[i] for i in idx],
                [self.wcs.cunit[i] for i in idx])
        return w

    def wcs_world2pix(self, *args):
        origin = args[-1]
        world = args[:-1]
        out = []
        for i, x in enumerate(world):
            x = np.asarray(x, dtype=float)
            out.append((x - self.wcs.crval[i]) / self.wcs.cdelt[i] + self.wcs.crpix[i] - 1 + origin)
        return out

    def wcs_pix2world(self, *args):
        origin = args[-1]
        pix = args[:-1]
        out = []
        for i, p in enumerate(pix):
            p = np.asarray(p, dtype=float)
            out.append(self.wcs.crval[i] + self.wcs.cdelt[i] * (p + 1 - origin - self.wcs.crpix[i]))
        return out

    def deepcopy(self):
        return _copy.deepcopy(self)


def skycoord_to_pixel(coords, wcs, origin=1, mode="wcs"):
    """SIN (orthographic) projection of ICRS directions to pixels: the inverse
    of ``pixel_to_skycoord``; NaN for directions behind the tangent plane.
    ``coords`` is a SkyCoord or a sequence of them; returns (x, y) arrays."""
    w = wcs.wcs
    items = coords if isinstance(coords, (list, tuple)) else [coords]
    ra0, dec0 = math.radians(w.crval[0]), math.radians(w.crval[1])
    xs, ys = [], []
    for c in items:
        ra, dec = c.ra.rad, c.dec.rad
        da = ra - ra0
        l = math.cos(dec) * math.sin(da)
        m = math.sin(dec) * math.cos(dec0) - math.cos(dec) * math.sin(dec0) * math.cos(da)
        n = math.sin(dec) * math.sin(dec0) + math.cos(dec) * math.cos(dec0) * math.cos(da)
        if n < 0.0:
            xs.append(float("nan"))
            ys.append(float("nan"))
            continue
        xs.append(l / math.radians(w.cdelt[0]) + w.crpix[0] - 1 + origin)
        ys.append(m / math.radians(w.cdelt[1]) + w.crpix[1] - 1 + origin)
    return np.array(xs), np.array(ys)


def pixel_to_skycoord(xp, yp, wcs, origin=1):
    """SIN (orthographic) deprojection of a pixel to an ICRS direction."""
    w = wcs.wcs
    x = math.radians(w.cdelt[0] * (xp - origin + 1 - w.crpix[0]))
    y = math.radians(w.cdelt[1] * (yp - origin + 1 - w.crpix[1]))
    l, m = x, y  # intermediate world coordinates are the direction cosines (l east)
    ra0, dec0 = math.radians(w.crval[0]), math.radians(w.crval[1])
    n = math.sqrt(max(0.0, 1.0 - l * l - m * m))
    dec = math.asin(m * math.cos(dec0) + n * math.sin(dec0))
    ra = ra0 + math.atan2(l, n * math.cos(dec0) - m * math.sin(dec0))
    return SkyCoord(ra, dec)


# ---------------------------------------------------------------------------
# Visibility
# ---------------------------------------------------------------------------
class _VisAcc:
    def __init__(self, vis):
        self._v = vis

    @property
    def polarisation_frame(self):
        return PolarisationFrame(self._v.attrs["_polarisation_frame"])

    @property
    def npol(self):
        return self.polarisation_frame.npol

    @property
    def nchan(self):
        return int(self._v._vars["frequency"].shape[0])

    @property
    def ntimes(self):
        return int(self._v._vars["time"].shape[0])

    @property
    def nbaselines(self):
        return int(self._v._vars["vis"].shape[1])

    @property
    def nants(self):
        b = np.asarray(self._v.attrs["baselines"])
        return int(b.max()) + 1 if b.size else 0

    def _mask(self):
        f = self._v._vars["flags"]
        return 1 - f

    @property
    def flagged_vis(self):
        return self._v._vars["vis"] * self._mask()

    @property
    def flagged_weight(self):
        return self._v._vars["weight"] * self._mask()

    @property
    def flagged_imaging_weight(self):
        return self._v._vars["imaging_weight"] * self._mask()

    @property
    def uvw_lambda(self):
        uvw = self._v._vars["uvw"]
        k = self._v._vars["frequency"] / C_M_S
        if torch is not None and isinstance(uvw, torch.Tensor):
            k = torch.as_tensor(k, device=uvw.device, dtype=uvw.dtype)
            return uvw[:, :, None, :] * k[None, None, :, None]
        return np.einsum("tbs,k->tbks", np.asarray(uvw), np.asarray(k)).view(_FlatCopyArray)

    @property
    def u(self):
        return _Derived(self._v._vars["uvw"][..., 0])

    @property
    def v(self):
        return _Derived(self._v._vars["uvw"][..., 1])

    @property
    def w(self):
        return _Derived(self._v._vars["uvw"][..., 2])

    def qa_visibility(self, context=None):
        avis = np.abs(np.asarray(_host(self._v._vars["vis"])))
        data = {"maxabs": float(avis.max()), "minabs": float(avis.min()), "rms": float(np.std(avis)),
                "medianabs": float(np.median(avis))}
        return _QA(data)


class _FlatCopyArray(np.ndarray):
    """ndarray whose ``.flat`` is a writable copy: the reference calls
    ``numpy.nan_to_num(uvw_lambda[..., chan, 0].flat)`` (gridding.py:49-55),
    which numpy >= 2 rejects on a flatiter."""

    @property
    def flat(self):
        return np.asarray(self).ravel().copy()


class _QA:
    def __init__(self, data):
        self.data = data


def _host(a):
    if torch is not None and isinstance(a, torch.Tensor):
        return a.detach().cpu().numpy()
    return a


class Visibility(Dataset):
    """Visibility with dims [time, baseline, frequency, polarisation]."""

    def groupby(self, coord, squeeze=False):
        """xarray's ``groupby("time", squeeze=False)`` as the sky-model
        drivers use it: (time, one-time-sample Visibility) pairs."""
        if coord != "time":
            raise ValueError(f"groupby: only 'time' is supported, not {coord}")
        times = np.asarray(self._vars["time"], dtype=float)
        times = np.unique(times[np.isfinite(times)])
        return list(zip(times.tolist(), visibility_time_slices(self)))

    @classmethod
    def constructor(cls, frequency=None, channel_bandwidth=None, phasecentre=None,
                    configuration=None, uvw=None, time=None, vis=None, weight=None,
                    integration_time=None, flags=None, baselines=None,
                    polarisation_frame=PolarisationFrame("stokesI"), source="anonymous",
                    meta=None, low_precision="float64", imaging_weight=None):
        vis_ = vis
        variables = {
            "vis": vis_,
            "uvw": uvw,
            "weight": weight if weight is not None else _ones_like(vis_, real=True),
            "imaging_weight": imaging_weight if imaging_weight is not None else (
                _clone(weight) if weight is not None else _ones_like(vis_, real=True)),
            "flags": flags if flags is not None else _zeros_int_like(vis_),
            "frequency": np.asarray(frequency, dtype=float),
            "channel_bandwidth": np.asarray(channel_bandwidth if channel_bandwidth is not None
                                            else np.ones(len(frequency)), dtype=float),
            "time": np.asarray(time, dtype=float),
            "integration_time": np.asarray(integration_time if integration_time is not None
                                           else np.ones(len(time)), dtype=float),
        }
        if hasattr(baselines, "data") and not isinstance(baselines, np.ndarray):
            baselines = baselines.data
        attrs = {
            "phasecentre": phasecentre,
            "configuration": configuration,
            "source": source,
            "meta": meta,
            "baselines": np.asarray(baselines) if baselines is not None else None,
            "_polarisation_frame": polarisation_frame.type if isinstance(
                polarisation_frame, PolarisationFrame) else polarisation_frame,
        }
        return cls(variables, attrs)

    @property
    def visibility_acc(self):
        return _VisAcc(self)

    @property
    def phasecentre(self):
        return self.attrs["phasecentre"]

    @property
    def configuration(self):
        return self.attrs["configuration"]

    @property
    def baselines(self):
        return _Plain(self.attrs["baselines"])

    def copy(self, deep=True, data=None, zero=False):
        return self._copy_with(deep=deep, zero_vars=("vis",) if zero else ())

    def sel(self, indexers=None, time=None):
        """Select a time slice (closed interval, as xarray's label slicing);
        accepts ``sel({"time": slice(a, b)})`` and ``sel(time=slice(a, b))``."""
        if isinstance(indexers, dict):
            time = indexers.get("time", time)
        t = np.asarray(self._vars["time"])
        mask = np.ones(len(t), dtype=bool)
        if time is not None:
            if time.start is not None:
                mask &= t >= time.start
            if time.stop is not None:
                mask &= t <= time.stop
        idx = np.nonzero(mask)[0]
        new = self._copy_with(deep=False)
        for k in ("vis", "uvw", "weight", "imaging_weight", "flags"):
            a = self._vars[k]
            if torch is not None and isinstance(a, torch.Tensor):
                new._vars[k] = a[torch.as_tensor(idx, device=a.device)]
            else:
                new._vars[k] = a[idx]
        new._vars["time"] = t[idx]
        new._vars["integration_time"] = np.asarray(self._vars["integration_time"])[idx]
        return new


class _Plain:
    def __init__(self, data):
        self.data = data


def _ones_like(v, real=False):
    if torch is not None and isinstance(v, torch.Tensor):
        return torch.ones(v.shape, device=v.device, dtype=torch.float64 if real else v.dtype)
    return np.ones(np.shape(v), dtype=float if real else np.asarray(v).dtype)


def _zeros_int_like(v):
    if torch is not None and isinstance(v, torch.Tensor):
        return torch.zeros(v.shape, device=v.device, dtype=torch.int32)
    return np.zeros(np.shape(v), dtype=int)


# ---------------------------------------------------------------------------
# Image
# ---------------------------------------------------------------------------
class _ImageAcc:
    def __init__(self, im):
        self._im = im

    @property
    def wcs(self):
        return self._im.attrs["wcs"]

    @property
    def polarisation_frame(self):
        return PolarisationFrame(self._im.attrs["_polarisation_frame"])

    @property
    def shape(self):
        return tuple(self._im._vars["pixels"].shape)

    @property
    def nchan(self):
        return self.shape[0]

    @property
    def npol(self):
        return self.shape[1]

    @property
    def phasecentre(self):
        w = self.wcs.wcs
        return SkyCoord(math.radians(w.crval[0]), math.radians(w.crval[1]))

    def is_canonical(self):
        w = self.wcs.wcs
        ok = len(self.shape) == 4 and w.ctype[0].startswith("RA") and w.ctype[1].startswith("DEC")
        ok = ok and w.ctype[2] == "STOKES" and w.ctype[3] == "FREQ"
        return bool(ok)

    def qa_image(self, context=None):
        d = np.asarray(_host(self._im._vars["pixels"]))
        return _QA({"max": float(d.max()), "min": float(d.min()), "maxabs": float(np.abs(d).max()),
                    "rms": float(d.std()), "sum": float(d.sum())})


class Image(Dataset):
    @classmethod
    def constructor(cls, data, polarisation_frame, wcs, clean_beam=None):
        return cls({"pixels": data},
                   {"wcs": wcs,
                    "_polarisation_frame": polarisation_frame.type if isinstance(
                        polarisation_frame, PolarisationFrame) else polarisation_frame,
                    "clean_beam": clean_beam})

    @property
    def image_acc(self):
        return _ImageAcc(self)

    def copy(self, deep=True, data=None, zero=False):
        """``data`` (xarray's copy(data=...)) becomes the copy's pixels as is."""
        return self._copy_with(deep=deep, zero_vars=("pixels",) if zero else (),
                               replace=None if data is None else {"pixels": data})


def create_image(npixel, cellsize, phasecentre, polarisation_frame=PolarisationFrame("stokesI"),
                 frequency=1.0e8, channel_bandwidth=1.0e6, nchan=1, dtype="float64"):
    """Canonical image: RA---SIN, DEC--SIN, STOKES, FREQ; cellsize in radians."""
    npol = polarisation_frame.npol
    wcs = WCS(4, ["RA---SIN", "DEC--SIN", "STOKES", "FREQ"],
              [npixel // 2 + 1, npixel // 2 + 1, 1.0, 1.0],
              [-math.degrees(cellsize), math.degrees(cellsize), 1.0, channel_bandwidth],
              [phasecentre.ra.deg, phasecentre.dec.deg, 1.0, frequency],
              ["deg", "deg", "", "Hz"])
    data = np.zeros([nchan, npol, npixel, npixel], dtype=dtype)
    return Image.constructor(data, polarisation_frame, wcs)


# ---------------------------------------------------------------------------
# GridData / ConvolutionFunction
# ---------------------------------------------------------------------------
class _GridAcc:
    def __init__(self, gd):
        self._g = gd

    @property
    def griddata_wcs(self):
        return self._g.attrs["grid_wcs"]

    @property
    def polarisation_frame(self):
        return PolarisationFrame(self._g.attrs["_polarisation_frame"])

    @property
    def shape(self):
        return tuple(self._g._vars["pixels"].shape)


class GridData(Dataset):
    @classmethod
    def constructor(cls, data, grid_wcs, polarisation_frame):
        return cls({"pixels": data}, {"grid_wcs": grid_wcs,
                                      "_polarisation_frame": polarisation_frame.type})

    @property
    def griddata_acc(self):
        return _GridAcc(self)

    def copy(self, deep=True, zero=False):
        return self._copy_with(deep=deep, zero_vars=("pixels",) if zero else ())


def create_griddata_from_image(im, polarisation_frame=None):
    """uv grid matching an image: cdelt_uv = 1/(npix * cell) (datamodels convention)."""
    nchan, npol, ny, nx = im["pixels"].data.shape
    iw = im.image_acc.wcs.wcs
    pf = polarisation_frame or im.image_acc.polarisation_frame
    d2r = math.pi / 180.0
    gw = WCS(4, ["UU", "VV", "STOKES", "FREQ"], [nx // 2 + 1, ny // 2 + 1, 1.0, 1.0],
             [1.0 / (nx * iw.cdelt[0] * d2r), 1.0 / (ny * iw.cdelt[1] * d2r), 1.0, iw.cdelt[3]],
             [0.0, 0.0, 1.0, iw.crval[3]])
    return GridData.constructor(np.zeros([nchan, pf.npol, ny, nx], dtype=complex), gw, pf)


class _CFAcc:
    def __init__(self, cf):
        self._c = cf

    @property
    def cf_wcs(self):
        return self._c.attrs["cf_wcs"]

    @property
    def polarisation_frame(self):
        return PolarisationFrame(self._c.attrs["_polarisation_frame"])

    @property
    def shape(self):
        return tuple(self._c._vars["pixels"].shape)


class ConvolutionFunction(Dataset):
    """Pixels [nchan, npol, nw, ndv, ndu, gv, gu]; cf_wcs axes (u, v, du, dv, w, stokes, freq)."""

    @classmethod
    def constructor(cls, data, cf_wcs, polarisation_frame):
        return cls({"pixels": data}, {"cf_wcs": cf_wcs,
                                      "_polarisation_frame": polarisation_frame.type})

    @property
    def convolutionfunction_acc(self):
        return _CFAcc(self)


# ---------------------------------------------------------------------------
# GainTable / SkyComponent
# ---------------------------------------------------------------------------
class _GTAcc:
    def __init__(self, gt):
        self._g = gt

    @property
    def nants(self):
        return self._g._vars["gain"].shape[1]

    @property
    def nchan(self):
        return self._g._vars["gain"].shape[2]

    @property
    def nrec(self):
        return self._g._vars["gain"].shape[3]

    @property
    def ntimes(self):
        return self._g._vars["gain"].shape[0]


class GainTable(Dataset):
    @classmethod
    def constructor(cls, gain, time, interval, weight, residual, frequency, receptor_frame,
                    phasecentre=None, configuration=None, jones_type="T"):
        return cls({"gain": gain, "weight": weight, "residual": residual,
                    "time": np.asarray(time, float), "interval": np.asarray(interval, float),
                    "frequency": np.asarray(frequency, float)},
                   {"receptor_frame": receptor_frame, "phasecentre": phasecentre,
                    "configuration": configuration, "jones_type": jones_type})

    @property
    def gaintable_acc(self):
        return _GTAcc(self)

    def copy(self, deep=True, zero=False):
        return self._copy_with(deep=deep)


def create_gaintable_from_visibility(vis, timeslice=None, jones_type="T"):
    """One gain row per time slot (``timeslice`` seconds, default every
    integration); nchan = 1 for T/G jones, = vis nchan for B."""
    times = np.asarray(vis.time.data)
    if timeslice is None or timeslice == "auto":
        gain_times = times.copy()
        interval = np.asarray(vis.integration_time.data, float).copy()
        if len(times) > 1:
            interval = np.full(len(times), float(np.min(np.diff(times))) if timeslice is None else 0.0)
            interval[:] = np.median(np.diff(times))
    else:
        nt = max(1, int(math.ceil((times.max() - times.min()) / timeslice)) if len(times) > 1 else 1)
        gain_times = times.min() + timeslice * (np.arange(nt) + 0.5)
        interval = np.full(nt, float(timeslice))
    nants = vis.visibility_acc.nants
    pf = vis.visibility_acc.polarisation_frame
    nrec = 1 if pf.npol == 1 else 2
    nchan = vis.visibility_acc.nchan if jones_type == "B" else 1
    freq = np.asarray(vis.frequency.data) if jones_type == "B" else np.array([np.mean(vis.frequency.data)])
    nt = len(gain_times)
    gain = np.zeros([nt, nants, nchan, nrec, nrec], dtype=complex)
    for r in range(nrec):
        gain[..., r, r] = 1.0
    weight = np.ones([nt, nants, nchan, nrec, nrec])
    residual = np.zeros([nt, nchan, nrec, nrec])
    rf = "stokesI" if nrec == 1 else ("linear" if pf.type.startswith("linear") else "circular")
    return GainTable.constructor(gain, gain_times, interval, weight, residual, freq,
                                 PolarisationFrame(rf) if rf != "stokesI" else PolarisationFrame("stokesI"),
                                 vis.phasecentre, vis.configuration, jones_type)


class SkyComponent:
    """Positional order of ska-sdp-datamodels: direction, frequency, name, flux."""

    def __init__(self, direction=None, frequency=None, name=None, flux=None, shape="Point",
                 polarisation_frame=PolarisationFrame("stokesIQUV"), params=None):
        self.direction = direction
        self.frequency = np.asarray(frequency, dtype=float)
        self.flux = np.asarray(flux)
        self.name = name
        self.shape = shape
        self.polarisation_frame = polarisation_frame
        self.params = params or {}

    @property
    def nchan(self):
        return self.flux.shape[0]

    @property
    def npol(self):
        return self.flux.shape[1]

    def copy(self):
        return _copy.deepcopy(self)


# ---------------------------------------------------------------------------
# SkyModel
# ---------------------------------------------------------------------------
class SkyModel:
    """image + point components + optional gain table and mask
    (ska-sdp-datamodels' SkyModel attributes used by the sky_model drivers)."""

    def __init__(self, image=None, components=None, gaintable=None, mask=None, fixed=False):
        self.image = image
        self.components = list(components) if components is not None else []
        self.gaintable = gaintable
        self.mask = mask
        self.fixed = fixed

    def copy(self):
        return _copy.deepcopy(self)


_TIME_VARS = ("vis", "uvw", "weight", "imaging_weight", "flags", "time", "integration_time")


def visibility_time_slices(vis):
    """One Visibility per distinct time value, in increasing time order, as
    xarray's ``vis.groupby("time", squeeze=False)`` yields them: the rows
    sharing a time value form one group (a view of the parent's arrays when
    they are consecutive, a gathered copy otherwise).  Rows whose time is not
    finite belong to no group, as xarray's groupby drops NaN labels."""
    times = np.asarray(vis._vars["time"], dtype=float)
    finite = np.isfinite(times)
    keys, inv = np.unique(times[finite], return_inverse=True)
    idx = np.flatnonzero(finite)
    order = np.argsort(inv, kind="stable")
    bounds = np.searchsorted(inv[order], np.arange(keys.size + 1))
    out = []
    for g in range(keys.size):
        rows = idx[order[bounds[g]:bounds[g + 1]]]
        if rows[-1] - rows[0] + 1 == rows.size:
            sel = slice(int(rows[0]), int(rows[-1]) + 1)
        else:
            sel = rows
        rep = {}
        for k in _TIME_VARS:
            if k not in vis._vars:
                continue
            a = vis._vars[k]
            if isinstance(sel, slice):
                rep[k] = a[sel]
            elif torch is not None and isinstance(a, torch.Tensor):
                rep[k] = a[torch.as_tensor(sel, device=a.device)]
            else:
                rep[k] = np.asarray(a)[sel]
        out.append(vis._copy_with(deep=False, replace=rep))
    return out
