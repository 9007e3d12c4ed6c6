"""Convolution-function (AW-projection) gridding on MI355X."""
from .gridding import (convolution_mapping_visibility, degrid_visibility_from_griddata,  # noqa: F401
                       fft_griddata_to_image, fft_image_to_griddata,
                       grid_visibility_to_griddata, spatial_mapping)
