"""Metric definitions: nominal inversion count 2 n^3 (LAPACK getrf+getri), and the
residual gate that decides whether a benchmarked inverse is correct.

The reference prints ``residual: ||A A^-1 - I||_inf`` after every run (main.cpp:490-507) but never
fails on it.  Here a wrong inverse must be a failure, not a fast success: ``bench.py`` exits 2 when
the residual is non-finite or fails the gate below (the CLI's ``--check-residual TOL`` is the
absolute form).

The gate is on the NORMALISED residual (LAPACK's inverse test ratio, xGET03)

    rho = ||A X - I||_inf / (||A||_inf ||X||_inf eps_dtype)       accept  rho <= RHO_PER_N * n

not on a per-(generator, size) absolute band.  The absolute residual of a correct inverse scales
with the conditioning of the particular matrix, and that moves by 10-100x between seeds and sizes
of the same generator (fp64 random, one seed: 1.3e-7 at N = 8192, 1.7e-5 at 16384, 2.6e-6 at
32768), so any band keyed on (gen, n) is either loose where the matrix is benign or a false failure
where it is not.  rho divides the conditioning out.  Measured rho / n on the host engine
(``bench/residual_ratio.py``, seeds 1-2, n = 100-1500, m = 8-128): fp64 random <= 0.13,
randshift <= 0.003, absdiff <= 0.47 (grows with m); fp32 random <= 0.035,
randshift <= 0.002, absdiff <= 0.014, hilbert <= 0.72 (kappa ~ 1e13+: the inverse is garbage but
its residual is still the backward-stable size).  GPU: ``profiles/residual_gate_r5.md``.
A wrong inverse gives rho ~ 1 / (||A|| ||X|| eps) (a zeroed or stale row: residual O(1)), 1e9-1e12
at the benchmark sizes, against a bound of 2n: the gate separates them by 5+ orders of magnitude
(tests/test_bench_cpu.py plants one with GJ_TEST_CORRUPT).
"""
from __future__ import annotations

import math
from typing import Optional

EPS = {"fp64": 2.220446049250313e-16, "fp32": 1.1920928955078125e-07}
RHO_PER_N = 2.0  # accepted rho / n: above every measured correct run (max 0.72) by >= 2.8x


def flops_nominal(n: int) -> float:
    return 2.0 * float(n) ** 3


def gflops_nominal(n: int, seconds: float) -> float:
    return flops_nominal(n) / seconds / 1e9 if seconds > 0 else 0.0


def residual_ratio(res: Optional[float], norm_a: float, norm_inv: float, dtype: str = "fp64") -> float:
    """rho = ||A X - I|| / (||A|| ||X|| eps) (inf-norms); inf when anything is non-finite or zero."""
    if res is None or not math.isfinite(res) or not (norm_a > 0 and norm_inv > 0) \
            or not math.isfinite(norm_a * norm_inv):
        return math.inf
    return res / (norm_a * norm_inv * EPS[dtype])


def residual_bound(n: int, norm_a: float, norm_inv: float, dtype: str = "fp64") -> float:
    """Largest ||A X - I||_inf accepted for a correct inverse of this matrix (absolute form of the
    gate: RHO_PER_N * n * ||A|| ||X|| eps)."""
    return RHO_PER_N * n * norm_a * norm_inv * EPS[dtype]


def residual_ok(res: Optional[float], n: int, norm_a: float, norm_inv: float, dtype: str = "fp64") -> bool:
    rho = residual_ratio(res, norm_a, norm_inv, dtype)
    return math.isfinite(rho) and rho <= RHO_PER_N * n
