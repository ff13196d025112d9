"""Pure-numpy oracle of the reference algorithm (fixed-bug semantics), used by the tests.

Implements Jordan() of the reference (main.cpp:953-1204) literally — physical block-row swaps,
separate B = I part, per-step normalisation — with the pivot-row bug at main.cpp:1095 fixed and the
pivot tie rule of SURVEY.md §4.3.4 (min ||inv||_inf, ties -> larger rank, then smaller local row).
It is deliberately a different formulation from the native engine (which never swaps rows and
inverts in place), so agreement is a real cross-check.
"""
from __future__ import annotations

import numpy as np

_MASK = (1 << 64) - 1


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(_MASK)
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(_MASK)
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(_MASK)
    return x ^ (x >> np.uint64(31))


def generate_matrix(n: int, kind: str = "absdiff", seed: int = 0) -> np.ndarray:
    """Same values as csrc/include/gj/gen.hpp (bitwise for 'random')."""
    i = np.arange(n, dtype=np.int64)[:, None]
    j = np.arange(n, dtype=np.int64)[None, :]
    if kind == "absdiff":
        return np.abs(i - j).astype(np.float64)
    if kind == "hilbert":
        return 1.0 / (i + j + 1).astype(np.float64)
    if kind == "identity":
        return np.eye(n)
    if kind == "randshift":  # random + sqrt(n) I (gen.hpp GenKind::RandomShifted)
        return generate_matrix(n, "random", seed) + np.sqrt(float(n)) * np.eye(n)
    if kind == "random":
        with np.errstate(over="ignore"):
            s = (np.uint64(seed) * np.uint64(0x2545F4914F6CDD1D)) & np.uint64(_MASK)
            key = s ^ (i.astype(np.uint64) << np.uint64(32)) ^ j.astype(np.uint64)
            h = _splitmix64(key)
        return (h >> np.uint64(11)).astype(np.float64) * (2.0 / 9007199254740992.0) - 1.0
    raise ValueError(kind)


def _block_inverse(P: np.ndarray, thresh: float):
    """Scalar GJ with partial pivoting (reference inverse_block, main.cpp:746-820)."""
    m = P.shape[0]
    a = P.copy()
    b = np.eye(m)
    for k in range(m):
        r = k + int(np.argmax(np.abs(a[k:, k])))
        if r != k:
            a[[k, r]] = a[[r, k]]
            b[[k, r]] = b[[r, k]]
        if not (abs(a[k, k]) >= thresh):
            return None
        piv = a[k, k]
        a[k, k + 1:] /= piv
        b[k] /= piv
        for i in range(m):
            if i != k:
                f = a[i, k]
                a[i, k + 1:] -= f * a[k, k + 1:]
                b[i] -= f * b[k]
    return b


def gauss_jordan_reference(A: np.ndarray, m: int, p: int = 1, eps: float = 1e-15):
    """Returns (inverse, pivots) where pivots[t] = logical block row chosen at step t, or raises
    ArithmeticError('singular matrix')."""
    A = np.asarray(A, dtype=np.float64)
    n = A.shape[0]
    Nr = -(-n // m)
    npad = Nr * m
    X = np.eye(npad)
    X[:n, :n] = A
    B = np.eye(npad)
    norm = np.abs(A).sum(axis=1).max()
    if abs(norm) < eps:
        raise ArithmeticError("singular matrix")
    thresh = eps * norm
    pivots = []
    for t in range(Nr):
        best = None
        for s in range(t, Nr):
            Y = _block_inverse(X[s * m:(s + 1) * m, t * m:(t + 1) * m], thresh)
            if Y is None:
                continue
            sc = np.abs(Y).sum(axis=1).max()
            if not np.isfinite(sc):
                continue
            key = (sc, -(s % p), s // p)
            if best is None or key < best[0]:
                best = (key, s, Y)
        if best is None:
            raise ArithmeticError("singular matrix")
        _, s, _ = best
        pivots.append(s)
        if s != t:
            rt, rs = slice(t * m, (t + 1) * m), slice(s * m, (s + 1) * m)
            X[rt], X[rs] = X[rs].copy(), X[rt].copy()
            B[rt], B[rs] = B[rs].copy(), B[rt].copy()
        rt = slice(t * m, (t + 1) * m)
        H = _block_inverse(X[rt, rt], thresh)
        X[rt] = H @ X[rt]
        B[rt] = H @ B[rt]
        for i in range(Nr):
            if i == t:
                continue
            ri = slice(i * m, (i + 1) * m)
            L = X[ri, rt].copy()
            X[ri] -= L @ X[rt]
            B[ri] -= L @ B[rt]
    return B[:n, :n], pivots
