"""Calibration hot path: solve_gaintable (batched StefCal on MI355X)."""
from .solvers import solve_gaintable  # noqa: F401
