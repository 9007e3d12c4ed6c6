"""MI355X-native predict/invert + calibration hot path of ska-sdp-func-python.

The reference-shaped API lives in the sub-packages that mirror the
reference's module layout (imaging, grid_data, calibration, visibility);
all compute goes through libska_sdp_hip.so (HIP for gfx950).
"""

__version__ = "0.1.0"
