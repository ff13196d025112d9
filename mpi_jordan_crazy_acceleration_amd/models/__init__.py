"""Solver "models": the block Gauss-Jordan inverter and the linear-system solver built on it."""
from .gauss_jordan import GaussJordan, inverse, run, solve  # noqa: F401
