"""Metric definitions: nominal inversion count 2 n^3 (LAPACK getrf+getri)."""


def flops_nominal(n: int) -> float:
    return 2.0 * float(n) ** 3


def gflops_nominal(n: int, seconds: float) -> float:
    return flops_nominal(n) / seconds / 1e9 if seconds > 0 else 0.0
