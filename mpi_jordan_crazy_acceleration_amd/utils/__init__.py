"""Utilities: numpy reference oracle, generators, flop accounting, timing."""
from .reference import gauss_jordan_reference, generate_matrix  # noqa: F401
from .metrics import gflops_nominal, residual_bound, residual_ok, residual_ratio  # noqa: F401
