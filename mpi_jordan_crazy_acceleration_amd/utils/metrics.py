"""Metric definitions: nominal inversion count 2 n^3 (LAPACK getrf+getri), and the
residual bounds that decide whether a benchmarked inverse is correct.

The reference prints ``residual: ||A A^-1 - I||_inf`` after every run (main.cpp:490-507) but never
fails on it.  Here a wrong inverse must be a failure, not a fast success: ``bench.py`` exits 2 when
the residual is non-finite or above ``residual_bound`` (the CLI's ``--check-residual TOL`` likewise).
The bounds sit 1-3 orders of magnitude above what correct runs measure, far below what a
wrong-but-finite inverse produces (the one unexplained bad run of round 3 had 1.9e4 against 4.8e-6;
a zeroed broadcast segment gives O(1) and above, tests/test_bench_cpu.py)."""
from __future__ import annotations

import math
from typing import Optional


def flops_nominal(n: int) -> float:
    return 2.0 * float(n) ** 3


def gflops_nominal(n: int, seconds: float) -> float:
    return flops_nominal(n) / seconds / 1e9 if seconds > 0 else 0.0


# (dtype, generator) -> (bound at n = 32768, exponent of n / 32768 it scales with).  Measured:
#   fp64 random   : 2.6e-6 at 32768 (BENCH_r03), 8.7e-11 at 1092, ~1e-10 at 300-1000 (CPU tier)
#   fp64 randshift: ~1e-12 (well conditioned at any n)
#   fp64 absdiff  : 4.5e-6 at 8192 / m = 60, grows with n and m
#   fp32 randshift: ~1e-4 (fp32 inverse, fp64 residual)
# Generators without an entry (hilbert: kappa ~ 1e16+, fp32 random: kappa eps32 >= 1 above 16384)
# are checked for finiteness only.
_BOUNDS = {
    ("fp64", "random"): (1e-4, 2.0),
    ("fp64", "randshift"): (1e-8, 1.0),
    ("fp64", "absdiff"): (1e-2, 2.0),
    ("fp32", "randshift"): (1e-1, 1.0),
}


def residual_bound(gen: str, n: int, dtype: str = "fp64") -> Optional[float]:
    """Largest ||A A^-1 - I||_inf accepted for a correct inverse (None: finiteness only)."""
    b = _BOUNDS.get((dtype, gen))
    if b is None:
        return None
    base, expo = b
    return base * max(1.0, (n / 32768.0) ** expo)


def residual_ok(res: Optional[float], gen: str, n: int, dtype: str = "fp64") -> bool:
    if res is None or not math.isfinite(res):
        return False
    bound = residual_bound(gen, n, dtype)
    return bound is None or res <= bound
