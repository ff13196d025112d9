"""Utilities: numpy reference oracle, generators, flop accounting, timing."""
from .reference import gauss_jordan_reference, generate_matrix  # noqa: F401
from .metrics import gflops_nominal  # noqa: F401
