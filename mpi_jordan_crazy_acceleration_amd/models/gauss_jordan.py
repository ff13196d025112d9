"""High-level single-process API of the block Gauss-Jordan inverter.

Mirrors the reference program's flow (``main.cpp:343-519``: build A, time ``Jordan``, print the
corners, recompute A, residual) but runs in-process: ``ranks`` host threads each drive one GPU
(RCCL between them when every rank has its own GPU) or one virtual host rank (``device="cpu"``).
For one process per GPU under ``torch.distributed`` use :class:`parallel.dist.DistributedGaussJordan`.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from .._native import load_native

STATUS = {0: "ok", 1: "singular matrix", 2: "not enough memory", 3: "cannot open", 4: "cannot read",
          5: "bad arguments", 6: "communication error", 7: "not enough memory for block",
          8: "verification failed"}


class SingularMatrixError(ArithmeticError):
    """Raised when every remaining candidate block is singular (reference: ``singular matrix``)."""


def _default_device() -> str:
    return "gpu" if load_native().device_count() > 0 else "cpu"


@dataclass
class GaussJordan:
    """Configuration of an in-process run (CLI-equivalent).

    block_size : reference ``m`` — the pivot block size (128 or 256 map best onto the MFMA tiles)
    ranks      : reference ``p`` — GPUs (device="gpu") or virtual host ranks (device="cpu")
    dtype      : "fp64" (reference) or "fp32" (CDNA4 fp32 MFMA path)
    """

    block_size: int = 128
    ranks: int = 1
    device: str = "auto"
    dtype: str = "fp64"
    comm: str = "auto"  # auto | rccl | loopback | async (stream-ordered virtual ranks)
    jitter_us: float = 0.0  # comm="async": random per-rank arrival delays (race screening)
    chunk_cols: int = 0
    depth: int = 0  # 0 = auto (engine.hpp)
    pivot: str = "block-min-inv-norm"  # or "partial" (block partial pivoting, SolveOptions::pivot)
    eps: float = 1e-15
    sync_debug: bool = False
    residual: str = "always"
    host_threads: int = 0
    race_check: bool = False  # happens-before schedule checker (RaceCheckDevice): report["races"]
    extra: dict = field(default_factory=dict)

    def _cfg(self, n: int) -> dict:
        dev = _default_device() if self.device == "auto" else self.device
        cfg = dict(n=int(n), m=int(self.block_size), ranks=int(self.ranks), device=dev,
                   dtype=self.dtype, comm=self.comm, chunk_cols=int(self.chunk_cols), depth=int(self.depth),
                   pivot=self.pivot,
                   eps=float(self.eps),
                   sync_debug=bool(self.sync_debug), residual=self.residual,
                   host_threads=int(self.host_threads), jitter_us=float(self.jitter_us),
                   race_check=bool(self.race_check))
        cfg.update(self.extra)
        return cfg

    def run(self, n: int, gen: str = "absdiff", seed: int = 0, file: Optional[str] = None,
            input: Optional[np.ndarray] = None, keep_inverse: bool = False, repeats: int = 1,
            rhs=None, keep_solution: bool = False, profile: bool = False) -> dict:
        """One CLI-equivalent run.  ``rhs``: None, "ones", "random", a file path, or an n-vector —
        then x = inv(A) b is computed on the devices and ``axb_residual`` = ||A x - b||_inf reported."""
        cfg = self._cfg(n)
        cfg.update(gen=gen, seed=int(seed), keep_inverse=keep_inverse, repeats=int(repeats),
                   keep_solution=bool(keep_solution), profile=bool(profile))
        if file is not None:
            cfg["file"] = str(file)
        if input is not None:
            cfg["input"] = np.ascontiguousarray(input, dtype=np.float64)
        if isinstance(rhs, str):
            cfg["rhs"] = rhs
        elif rhs is not None:
            cfg["rhs_input"] = np.ascontiguousarray(np.asarray(rhs, dtype=np.float64).reshape(-1))
        rep = load_native().run_local(cfg)
        rep["status_name"] = STATUS.get(rep["status"], "error")
        return rep

    def inverse(self, A):
        is_torch = isinstance(A, torch.Tensor)
        if is_torch and A.is_cuda and self.ranks == 1 and self.device in ("auto", "gpu"):
            return self._inverse_resident(A)
        a = A.detach().to("cpu", torch.float64).numpy() if is_torch else np.asarray(A, dtype=np.float64)
        if a.ndim != 2 or a.shape[0] != a.shape[1]:
            raise ValueError("A must be square")
        rep = self.run(a.shape[0], input=a, keep_inverse=True)
        if rep["status"] == 1:
            raise SingularMatrixError("singular matrix")
        if rep["status"] != 0:
            raise RuntimeError(rep["message"] or rep["status_name"])
        inv = rep["inverse"]
        if is_torch:
            return torch.from_numpy(inv).to(device=A.device, dtype=A.dtype)
        return inv


    def _engine_resident(self, A: torch.Tensor):
        """The native engine, solved on a CUDA tensor's rows (copied device-to-device)."""
        if A.ndim != 2 or A.shape[0] != A.shape[1]:
            raise ValueError("A must be square")
        C = load_native()
        tdt = torch.float64 if self.dtype == "fp64" else torch.float32
        a = A.detach().to(tdt).contiguous()
        n = a.shape[0]
        idx = a.device.index if a.device.index is not None else torch.cuda.current_device()
        eng = C.Engine(_hip_device(idx), C.self_comm(), n, int(self.block_size), self.dtype,
                       int(self.chunk_cols), float(self.eps), bool(self.sync_debug), int(self.depth),
                       pivot=self.pivot)
        torch.cuda.synchronize(a.device)  # A may have been written on torch's stream
        eng.upload_rows_device(a.data_ptr(), a.stride(0))
        st = eng.solve()
        if st["status"] == 1:
            raise SingularMatrixError("singular matrix")
        if st["status"] != 0:
            raise RuntimeError(STATUS.get(st["status"], "error"))
        return eng, a

    def _inverse_resident(self, A: torch.Tensor) -> torch.Tensor:
        """Inverse of a CUDA tensor without host round trips: the rows are copied device-to-device
        into the engine's panel and the result straight back into a new tensor on A's device."""
        eng, a = self._engine_resident(A)
        out = torch.empty_like(a)
        eng.download_rows_device(out.data_ptr(), out.stride(0))
        return out.to(A.dtype)

    def solve_resident(self, A: torch.Tensor, b, max_refine: int = -1, tol: float = 1e-15):
        """A x = b for a CUDA tensor A through the engine (Engine::solve_rhs_device): x = inv(A) b by
        the native GEMV, then iterative refinement with the residual b - A x in fp64 against A's
        rows (an fp32 inverse refines to fp64 accuracy on a well-conditioned system, as the CLI's
        --rhs path).  b: an n-vector or an n x k matrix (columns refined one by one).  Returns
        (x on A's device in A's dtype, info per column)."""
        eng, _ = self._engine_resident(A)
        a64 = A.detach().to(torch.float64).contiguous()
        torch.cuda.synchronize(a64.device)
        bt = b.detach().to("cpu", torch.float64) if isinstance(b, torch.Tensor) else \
            torch.as_tensor(np.asarray(b, dtype=np.float64))
        cols = bt.reshape(bt.shape[0], -1).numpy()
        xs, infos = [], []
        for j in range(cols.shape[1]):
            x, info = eng.solve_rhs_device(np.ascontiguousarray(cols[:, j]), a64.data_ptr(), a64.stride(0),
                                           int(max_refine), float(tol))
            xs.append(x)
            infos.append(info)
        x = np.stack(xs, axis=1).reshape(bt.shape)
        return torch.from_numpy(x).to(device=A.device, dtype=A.dtype), infos


_HIP_DEVICES: dict = {}


def _hip_device(idx: int):
    if idx not in _HIP_DEVICES:
        _HIP_DEVICES[idx] = load_native().hip_device(idx)
    return _HIP_DEVICES[idx]


def inverse(A, block_size: int = 128, **kw):
    """Inverse of a dense square matrix by block Gauss-Jordan (reference semantics, fixed pivot bug)."""
    return GaussJordan(block_size=block_size, residual="never", **kw).inverse(A)


def solve(A, b, block_size: int = 128, **kw):
    """Solve ``A x = b`` via the block Gauss-Jordan inverse.

    A single right-hand side runs the native path (x = inv(A) b on the devices, the GEMV next to
    the inverse's rows, refined in fp64); a matrix of right-hand sides multiplies by the returned
    inverse on the host path.  A CUDA tensor A stays on its GPU: the engine solves it in place and
    every right-hand side (vector or matrix columns) goes through Engine::solve_rhs_device, the
    native GEMV plus fp64 refinement (never a bare ``inv @ b``)."""
    is_torch = isinstance(A, torch.Tensor)
    if is_torch and A.is_cuda:
        gj = GaussJordan(block_size=block_size, residual="never", **kw)
        x, _ = gj.solve_resident(A, b)
        return x
    bn = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b, dtype=np.float64)
    if bn.ndim == 1:
        a = A.detach().to("cpu", torch.float64).numpy() if is_torch else np.asarray(A, dtype=np.float64)
        gj = GaussJordan(block_size=block_size, residual="never", **kw)
        rep = gj.run(a.shape[0], input=a, rhs=bn, keep_solution=True)
        if rep["status"] == 1:
            raise SingularMatrixError("singular matrix")
        if rep["status"] != 0:
            raise RuntimeError(rep["message"] or rep["status_name"])
        x = rep["x"].reshape(-1)
        return torch.from_numpy(x).to(device=A.device, dtype=A.dtype) if is_torch else x
    inv = inverse(A, block_size=block_size, **kw)
    if isinstance(inv, torch.Tensor):
        return inv @ (b if isinstance(b, torch.Tensor) else torch.as_tensor(b, dtype=inv.dtype))
    return inv @ np.asarray(b, dtype=np.float64)


def run(n: int, m: int, ranks: int = 1, device: str = "auto", gen: str = "absdiff", seed: int = 0,
        file: Optional[str] = None, dtype: str = "fp64", residual: str = "always", **kw) -> dict:
    """The reference CLI flow in-process; returns the report dict (glob_time, residual, corners...)."""
    return GaussJordan(block_size=m, ranks=ranks, device=device, dtype=dtype, residual=residual,
                       **kw).run(n, gen=gen, seed=seed, file=file)
