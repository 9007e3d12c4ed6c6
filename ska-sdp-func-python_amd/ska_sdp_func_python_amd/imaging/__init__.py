"""Imaging hot path: predict/invert (w-stacking NUFFT), the sky-component DFT and imaging weights."""
from .base import normalise_sumwt, shift_vis_to_image  # noqa: F401
from .dft import dft_skycomponent_visibility, extract_direction_and_flux  # noqa: F401
from .imaging import invert_visibility, predict_visibility  # noqa: F401
from .ng import invert_ng, predict_ng  # noqa: F401
from .weighting import (taper_visibility_gaussian, taper_visibility_tukey,  # noqa: F401
                        weight_visibility)
