"""Test configuration: import paths, the ``gpu`` marker and fixture loaders.

``-m "not gpu"`` (CPU, the build container): oracle restatements against the
reference-generated fixtures in tests/golden/, host-side logic, library
load/exports, and the world_size-2 gloo sharding test.
``-m gpu`` (MI355X): parity of the HIP path through the C ABI.
"""

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


def golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


@pytest.fixture
def load_golden():
    return golden


def rel_rms(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return float(np.sqrt(np.mean(np.abs(a - b) ** 2)) / max(np.sqrt(np.mean(np.abs(b) ** 2)), 1e-300))


def weight_case(g):
    """Flat arrays + grid geometry of a tests/golden/weight_*.npz fixture, with
    the model image / GridData rebuilt through the datamodels shim exactly as
    make_golden.make_weighting built them."""
    from ska_sdp_func_python_amd import datamodels as dm
    pf = dm.PolarisationFrame(str(g["pol_frame"]))
    npix, cell = int(g["npix"]), float(g["cell"])
    model = dm.create_image(npix, cell, dm.SkyCoord(0, -0.5), polarisation_frame=pf,
                            frequency=float(g["model_freq"]), channel_bandwidth=float(g["model_bw"]),
                            nchan=int(g["model_nchan"]))
    gd = dm.create_griddata_from_image(model, polarisation_frame=pf)
    gw = gd.griddata_acc.griddata_wcs.wcs
    wcs = ((gw.crval[0], gw.cdelt[0], gw.crpix[0]), (gw.crval[1], gw.cdelt[1], gw.crpix[1]))
    v2i = np.round(gd.griddata_acc.griddata_wcs.sub([4]).wcs_world2pix(g["freq"], 0)[0]).astype(int)
    nt, nb, nchan, npol = g["weight"].shape
    mask = 1 - g["flags"]
    return dict(uvw=g["uvw"].reshape(-1, 3), freq=g["freq"],
                fwt=(g["weight"] * mask).reshape(nt * nb, nchan, npol),
                fimw=(g["imaging_weight"] * mask).reshape(nt * nb, nchan, npol),
                vis_to_im=v2i, wcs=wcs, g_nchan=int(g["model_nchan"]), ny=npix, nx=npix,
                shape=(nt, nb, nchan, npol), model=model, pf=pf)
