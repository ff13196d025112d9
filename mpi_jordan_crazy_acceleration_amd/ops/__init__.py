"""Kernel-level wrappers of the hand-written gfx950 kernels, on torch tensors.

These call straight into the native kernels (no PyTorch fallback): a CUDA(HIP) tensor runs the HIP
kernel, a CPU tensor runs the host reference executor — chosen by the tensor's device, never
silently.  Used by the per-kernel numerics tests and for profiling single kernels.
"""
from __future__ import annotations

import functools

import torch

from .._native import load_native

_DT = {torch.float64: "fp64", torch.float32: "fp32"}


@functools.lru_cache(maxsize=None)
def _hip(idx: int):
    return load_native().hip_device(idx)


@functools.lru_cache(maxsize=None)
def _host():
    return load_native().host_device(0)


def device_for(t: torch.Tensor):
    if t.is_cuda:
        torch.cuda.synchronize(t.device)
        return _hip(t.device.index if t.device.index is not None else torch.cuda.current_device())
    return _host()


def _p(t: torch.Tensor) -> int:
    return t.data_ptr()


def gemm(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, op: str = "acc", a_kmajor: bool = False,
         zero_cols=(0, 0), zero_rows=(), zero_row_height: int = 0, tneg: torch.Tensor = None,
         latency: bool = False, dense: bool = False, c_in: torch.Tensor = None, row_blocks=None,
         row_block_m: int = 0, skip_cols=(0, 0)) -> torch.Tensor:
    """C += A@B (op="acc") or C = A@B (op="store").  With a_kmajor, ``A`` is given as A^T (K x M).

    Elimination extras (op="acc"): C enters as 0 in the columns ``zero_cols`` = (c0, c1) and in the
    row blocks [r, r + zero_row_height) for r in ``zero_rows`` (at most 8).  ``tneg`` (Nt x M view,
    Nt <= N, unit column stride): also receives -C^T of C's first Nt columns, the multiplier panel
    the engine's column / look-ahead updates write as they store C.  ``latency``: the small-tile
    launch the pivot chain uses.  ``dense``: the 5-workgroups-per-CU build of the fp64 LDS-DMA
    trailing update (the engine's choice under a CU reservation).  ``c_in`` (op="acc"): the
    accumulator's input array instead of C itself (C = c_in + A@B).  ``row_blocks`` with
    ``row_block_m``: only those row blocks of C / A^T take part (GemmExtra::rsel); M = C's rows is
    then the physical height and the product runs over len(row_blocks) * row_block_m rows.
    ``skip_cols`` = (s0, s1): those output columns are neither read nor written (GemmExtra::skip_c0
    / skip_c1; multiples of 128 on the GPU)."""
    assert A.dtype == B.dtype == C.dtype and A.stride(-1) == 1 and B.stride(-1) == 1 and C.stride(-1) == 1
    M, N = C.shape
    K = A.shape[0] if a_kmajor else A.shape[1]
    tp, ldt, tcols = 0, 0, 0
    if tneg is not None:
        assert tneg.dtype == C.dtype and tneg.shape[1] == M and 0 < tneg.shape[0] <= N and tneg.stride(-1) == 1
        tp, ldt, tcols = _p(tneg), tneg.stride(0), tneg.shape[0]
    cp, ldci = 0, 0
    if c_in is not None:
        assert c_in.dtype == C.dtype and c_in.shape == C.shape and c_in.stride(-1) == 1
        cp, ldci = _p(c_in), c_in.stride(0)
    rb = [int(b) for b in (row_blocks or [])]
    Msel = len(rb) * int(row_block_m) if row_block_m else M
    device_for(C).gemm(_DT[C.dtype], op, a_kmajor, Msel, N, K, _p(A), A.stride(0), _p(B), B.stride(0), _p(C),
                       C.stride(0), int(zero_cols[0]), int(zero_cols[1]), [int(r) for r in zero_rows],
                       int(zero_row_height), tp, ldt, bool(latency), tcols, bool(dense), cp, ldci, rb,
                       int(row_block_m), int(skip_cols[0]), int(skip_cols[1]))
    return C


def gemm_batch(products) -> None:
    """Independent small products in one launch: each item is (op, At, B, C) with At = A^T (K x M),
    op "acc" (C += A@B) or "store" (C = A@B).  All tensors share one dtype and device."""
    if not products:
        return
    C0 = products[0][3]
    descs = []
    for op, At, B, C in products:
        assert At.dtype == B.dtype == C.dtype == C0.dtype and At.stride(-1) == 1 and B.stride(-1) == 1
        assert C.stride(-1) == 1
        M, N = C.shape
        descs.append((op, M, N, At.shape[0], _p(At), At.stride(0), _p(B), B.stride(0), _p(C), C.stride(0)))
    device_for(C0).gemm_batch(_DT[C0.dtype], descs)


def generate(X: torch.Tensor, n: int, m: int, p: int = 1, k: int = 0, kind: str = "absdiff", seed: int = 0) -> torch.Tensor:
    device_for(X).generate(_DT[X.dtype], _p(X), n, m, p, k, kind, seed)
    return X


def extract_neg_t(X: torch.Tensor, col0: int, m: int) -> torch.Tensor:
    rows = X.shape[0]
    Lt = torch.empty((m, rows), dtype=X.dtype, device=X.device)
    device_for(X).extract_neg_t(_DT[X.dtype], _p(Lt), rows, _p(X), X.stride(0), rows, col0, m)
    return Lt


def block_inverse(Lt: torch.Tensor, n: int, m: int, p: int = 1, k: int = 0, used: torch.Tensor = None,
                  thresh: float = 0.0, nlive: int = -1):
    """Batched candidate inversion over the K-major multiplier panel Lt (m x rows).

    nlive >= 0: launch one workgroup per unused candidate only (the engine's form; scores / valid
    of used blocks are then left untouched), -1: one per local block.  Returns (inv_t [nblk, m, m] with inv_t[b] = inv(W_b)^T, scores [nblk], valid [nblk])."""
    nblk = Lt.shape[1] // m
    dev = Lt.device
    inv_t = torch.zeros((max(nblk, 1), m, m), dtype=Lt.dtype, device=dev)
    scores = torch.zeros(max(nblk, 1), dtype=torch.float64, device=dev)
    valid = torch.zeros(max(nblk, 1), dtype=torch.int32, device=dev)
    Nr = (n + m - 1) // m
    if used is None:
        used = torch.zeros(Nr, dtype=torch.int32, device=dev)
    device_for(Lt).block_inverse(_DT[Lt.dtype], _p(Lt), Lt.stride(0), _p(inv_t), _p(scores), _p(valid), _p(used),
                                 n, m, p, k, thresh, nlive)
    return inv_t[:nblk], scores[:nblk], valid[:nblk]


def permute_blocks(X: torch.Tensor, m: int, dst_blk: torch.Tensor, colsrc: torch.Tensor) -> torch.Tensor:
    rows, ncols = X.shape
    nblk, Nr = rows // m, ncols // m
    out = torch.empty_like(X)
    device_for(X).permute_blocks(_DT[X.dtype], _p(out), out.stride(0), _p(X), X.stride(0), nblk, m, Nr,
                                 _p(dst_blk), _p(colsrc))
    return out


def row_abs_max(X: torch.Tensor, n: int, m: int, p: int = 1, k: int = 0) -> float:
    out = torch.zeros(1, dtype=torch.float64, device=X.device)
    device_for(X).row_abs_max(_DT[X.dtype], _p(X), X.stride(0), n, m, p, k, _p(out))
    return float(out.item())


def residual(A_loc: torch.Tensor, Full: torch.Tensor, n: int, m: int, p: int = 1, k: int = 0) -> float:
    out = torch.zeros(1, dtype=torch.float64, device=A_loc.device)
    device_for(A_loc).residual(_DT[A_loc.dtype], _p(A_loc), _p(Full), n, m, p, k, _p(out))
    return float(out.item())
