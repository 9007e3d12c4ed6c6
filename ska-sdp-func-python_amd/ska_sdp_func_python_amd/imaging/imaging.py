"""Context dispatch (reference src/ska_sdp_func_python/imaging/imaging.py:28-105).

"ng" (default), "2d" (ng without w-stacking), "wg" (the reference's WAGG GPU
twin, same contract) and "hip" all run the HIP w-stacking NUFFT;
"awprojection" runs the HIP convolution-function gridder.  Unknown contexts
raise ValueError as in the reference.
"""

from .base import invert_awprojection, predict_awprojection
from .ng import invert_ng, predict_ng


def predict_visibility(vis, model, context="ng", gcfcf=None, **kwargs):
    if context == "awprojection":
        return predict_awprojection(vis, model, gcfcf=gcfcf)
    if context == "2d":
        return predict_ng(vis, model, do_wstacking=False, **kwargs)
    if context in ("ng", "wg", "hip"):
        return predict_ng(vis, model, **kwargs)
    raise ValueError(f"Unknown imaging context {context}")


def invert_visibility(vis, im, dopsf=False, normalise=True, context="ng", gcfcf=None, **kwargs):
    if context == "awprojection":
        return invert_awprojection(vis, im, dopsf=dopsf, normalise=normalise, gcfcf=gcfcf)
    if context == "2d":
        return invert_ng(vis, im, dopsf=dopsf, normalise=normalise, do_wstacking=False, **kwargs)
    if context in ("ng", "wg", "hip"):
        return invert_ng(vis, im, dopsf=dopsf, normalise=normalise, **kwargs)
    raise ValueError(f"Unknown imaging context {context}")
