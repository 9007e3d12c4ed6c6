"""Coordinate helpers used on the hot path (reference src/ska_sdp_func_python/util/)."""
