"""Calibration hot path: solve_gaintable (batched StefCal on MI355X) and apply_gaintable."""
from .operations import apply_gaintable  # noqa: F401
from .solvers import solve_gaintable  # noqa: F401
