"""apply_beam_to_skycomponent (reference
src/ska_sdp_func_python/sky_component/operations.py:366-444).

Host logic over a handful of components: each point component's flux is
multiplied (or, with ``inverse`` and a non-zero beam, divided) by the beam
pixel its direction projects to (SIN projection, origin 1, Python's
round-half-even); components off the image get zero flux.
"""

import collections.abc
import copy
import logging

import numpy as np

from ..datamodels import SkyComponent, skycoord_to_pixel

log = logging.getLogger("func-python-logger")


def apply_beam_to_skycomponent(sc, beam, phasecentre=None, inverse=False):
    single = not isinstance(sc, collections.abc.Iterable)
    if single:
        sc = [sc]
    ny = beam["pixels"].data.shape[2]
    nx = beam["pixels"].data.shape[3]
    pixels = beam["pixels"].data
    pixels = pixels.cpu().numpy() if hasattr(pixels, "cpu") else np.asarray(pixels)
    log.debug("apply_beam_to_skycomponent: Processing %d components", len(sc))
    wcs = beam.image_acc.wcs
    if wcs.wcs.ctype[0] != "RA---SIN":
        wcs = copy.deepcopy(wcs)
        wcs.wcs.ctype[0] = "RA---SIN"
        wcs.wcs.ctype[1] = "DEC--SIN"
        wcs.wcs.crval[0] = phasecentre.ra.deg
        wcs.wcs.crval[1] = phasecentre.dec.deg
    pixlocs = skycoord_to_pixel([c.direction for c in sc], wcs, origin=1, mode="wcs")
    newsc = []
    total_flux = np.zeros_like(sc[0].flux)
    for icomp, comp in enumerate(sc):
        assert comp.shape == "Point", f"Cannot handle shape {comp.shape}"
        pixloc = (pixlocs[0][icomp], pixlocs[1][icomp])
        if not np.isnan(pixloc).any():
            x, y = int(round(float(pixloc[0]))), int(round(float(pixloc[1])))
            if 0 <= x < nx and 0 <= y < ny:
                if inverse and (pixels[:, :, y, x] != 0.0).all():
                    comp_flux = comp.flux / pixels[:, :, y, x]
                else:
                    comp_flux = comp.flux * pixels[:, :, y, x]
                total_flux += comp_flux
            else:
                comp_flux = 0.0 * comp.flux
            newsc.append(SkyComponent(comp.direction, comp.frequency, comp.name, comp_flux,
                                      shape=comp.shape, polarisation_frame=comp.polarisation_frame))
    log.debug("apply_beam_to_skycomponent: %d components with total flux %s", len(newsc),
              total_flux)
    if single:
        return newsc[0]
    return newsc
