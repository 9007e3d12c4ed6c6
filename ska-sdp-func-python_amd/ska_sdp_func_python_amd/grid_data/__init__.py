"""Convolution-function (AW-projection) gridding and imaging-weight gridding on MI355X."""
from .gridding import (convolution_mapping_visibility, degrid_visibility_from_griddata,  # noqa: F401
                       fft_griddata_to_image, fft_image_to_griddata,
                       grid_visibility_to_griddata, grid_visibility_weight_to_griddata,
                       griddata_merge_weights, griddata_visibility_reweight, spatial_mapping)
