"""Closed-form coordinate transforms used by the hot path.

Restates reference ``src/ska_sdp_func_python/util/coordinate_support.py``
for the functions the predict/invert/DFT path touches, without astropy:
``skycoord_to_lmn`` (:436-460, l eastwards, returns n-1 as the reference's
``dc.x - 1``), ``xyz_to_uvw`` / ``uvw_to_xyz`` (:335-393) and
``lmn_to_skycoord`` (:463-490).
"""

import math

import numpy as np

from ..datamodels import SkyCoord


def skycoord_to_lmn(pos, phasecentre):
    """(l, m, n-1) of ``pos`` relative to ``phasecentre`` (radians)."""
    a, d = pos.ra.rad, pos.dec.rad
    a0, d0 = phasecentre.ra.rad, phasecentre.dec.rad
    da = a - a0
    l = math.cos(d) * math.sin(da)
    m = math.sin(d) * math.cos(d0) - math.cos(d) * math.sin(d0) * math.cos(da)
    n = math.sin(d) * math.sin(d0) + math.cos(d) * math.cos(d0) * math.cos(da)
    return l, m, n - 1.0


def lmn_to_skycoord(lmn, phasecentre):
    l, m = float(lmn[0]), float(lmn[1])
    n = math.sqrt(max(0.0, 1.0 - l * l - m * m))
    a0, d0 = phasecentre.ra.rad, phasecentre.dec.rad
    dec = math.asin(m * math.cos(d0) + n * math.sin(d0))
    ra = a0 + math.atan2(l, n * math.cos(d0) - m * math.sin(d0))
    return SkyCoord(ra, dec)


def xyz_to_uvw(xyz, ha, dec):
    """Rotate earth-frame (x, y, z) to (u, v, w) for hour angle / declination."""
    x, y, z = np.hsplit(np.asarray(xyz, dtype=float), 3)
    u = x * np.cos(ha) - y * np.sin(ha)
    v0 = x * np.sin(ha) + y * np.cos(ha)
    w = z * np.sin(dec) - v0 * np.cos(dec)
    v = z * np.cos(dec) + v0 * np.sin(dec)
    return np.hstack([u, v, w])


def uvw_to_xyz(uvw, ha, dec):
    u, v, w = np.hsplit(np.asarray(uvw, dtype=float), 3)
    v0 = v * np.sin(dec) - w * np.cos(dec)
    z = v * np.cos(dec) + w * np.sin(dec)
    x = u * np.cos(ha) + v0 * np.sin(ha)
    y = -u * np.sin(ha) + v0 * np.cos(ha)
    return np.hstack([x, y, z])
