"""Builders shared by the GPU tests (fixture arrays -> datamodels shim objects)."""

import numpy as np

from ska_sdp_func_python_amd import datamodels as dm


def vis_from_arrays(uvw, freq, vis, weight=None, flags=None, baselines=None, pf="stokesI",
                    times=None, phasecentre=None, integration_time=None):
    nt, nb = uvw.shape[:2]
    if baselines is None:
        baselines = np.stack(np.triu_indices(64, 1), 1)[:nb]
    shape = vis.shape
    times = np.arange(nt, dtype=float) if times is None else times
    return dm.Visibility.constructor(
        frequency=np.asarray(freq, float), channel_bandwidth=np.full(len(freq), 1e6),
        phasecentre=phasecentre or dm.SkyCoord(0.0, -0.8), uvw=uvw, time=times,
        vis=vis, weight=np.ones(shape) if weight is None else weight,
        flags=np.zeros(shape, int) if flags is None else flags, baselines=baselines,
        polarisation_frame=dm.PolarisationFrame(pf), integration_time=integration_time)
