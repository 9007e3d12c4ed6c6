"""Visibility helpers on the hot path (reference src/ska_sdp_func_python/visibility/)."""
from .base import calculate_visibility_phasor, phaserotate_visibility  # noqa: F401
from .operations import concatenate_visibility, divide_visibility  # noqa: F401
