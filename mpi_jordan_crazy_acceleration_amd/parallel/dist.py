"""One rank per process over ``torch.distributed`` (the MI355X deployment model).

* backend ``nccl`` (= RCCL on ROCm): each process drives ``cuda:LOCAL_RANK`` with the native
  HipDevice; the engine builds its own two RCCL communicators (one per issuing stream role) from
  unique ids broadcast through the default process group, and talks RCCL directly from C++ — no
  Python in the per-step path.
* backend ``gloo`` (CPU): the native HostDevice executes and collectives trampoline into
  ``torch.distributed`` via :class:`TorchDistComm` — the CPU-testable form of the same protocol.

Reference parity: this replaces MPI_Init/Comm_size/Comm_rank (main.cpp:65-93) and the per-rank
``solve`` driver (main.cpp:343-519).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .._native import load_native
from .layout import Layout, global_rows


class TorchDistComm:
    """Host-memory collectives for the native engine, implemented with torch.distributed (gloo)."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)

    @staticmethod
    def _view(addr: int, nbytes: int) -> torch.Tensor:
        if nbytes == 0:
            return torch.empty(0, dtype=torch.uint8)
        buf = (ctypes.c_char * nbytes).from_address(addr)
        return torch.frombuffer(buf, dtype=torch.uint8)

    def allgather(self, send: int, recv: int, nbytes: int) -> None:
        s = self._view(send, nbytes).clone()
        out = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
        dist.all_gather(out, s, group=self.group)
        self._view(recv, nbytes * self.world).copy_(torch.cat(out))

    def bcast(self, addr: int, nbytes: int, root: int) -> None:
        t = self._view(addr, nbytes)
        tmp = t.clone()
        dist.broadcast(tmp, src=root, group=self.group)
        t.copy_(tmp)

    def allreduce_max(self, addr: int, count: int) -> None:
        t = self._view(addr, count * 8)
        tmp = t.clone().view(torch.float64)
        dist.all_reduce(tmp, op=dist.ReduceOp.MAX, group=self.group)
        t.copy_(tmp.view(torch.uint8))

    def group_p2p(self, ops) -> None:
        reqs, recvs = [], []
        tags = {}
        for addr, nbytes, peer, is_send in ops:
            key = (peer, bool(is_send))
            tag = tags.get(key, 0)
            tags[key] = tag + 1
            if is_send:
                reqs.append(dist.isend(self._view(addr, nbytes).clone(), dst=peer, group=self.group, tag=tag))
            else:
                buf = torch.empty(nbytes, dtype=torch.uint8)
                reqs.append(dist.irecv(buf, src=peer, group=self.group, tag=tag))
                recvs.append((addr, nbytes, buf))
        for r in reqs:
            r.wait()
        for addr, nbytes, buf in recvs:
            self._view(addr, nbytes).copy_(buf)

    def barrier(self) -> None:
        dist.barrier(group=self.group)

    def host_max(self, v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())


def agree_comm_mode(group=None, need: Optional[int] = None) -> dict:
    """Collective: the RCCL communicator schedule every rank will use.

    Two communicators (SIDE: pivot records and panel pieces; COMM: row segments) let the pivot chain
    run ahead of the chunk broadcasts, but their progress argument needs them on different in-order
    hardware queues (README "Progress of the two communicators"), i.e. ``need`` (16) queues per
    process.  When any rank has fewer (HIP initialised before the package could raise
    GPU_MAX_HW_QUEUES, see runtime_env.effective_hw_queues), or any rank sets ``GJ_ONE_COMM=1``,
    EVERY rank takes the one-communicator schedule (RcclComm one_comm: one program order of
    collectives, safe on shared queues) -- a slower run, never a refusal and never a hang.  The
    decision is agreed here, before any RCCL communicator exists, because creating the second
    communicator is itself collective (reference: collective agreement, main.cpp:371-381).

    Returns ``{"one_comm": bool, "hw_queues": min over ranks, "reason": str}``."""
    from ..runtime_env import MIN_HW_QUEUES, effective_hw_queues

    need = MIN_HW_QUEUES if need is None else need
    rank = dist.get_rank(group)
    forced = os.environ.get("GJ_ONE_COMM", "0") not in ("", "0")
    mine = (effective_hw_queues(rank), forced)
    every = [None] * dist.get_world_size(group)
    dist.all_gather_object(every, mine, group=group)
    low = min(q for q, _ in every)
    short = [r for r, (q, _) in enumerate(every) if q < need]
    asked = [r for r, (_, f) in enumerate(every) if f]
    if short:
        reason = (f"rank(s) {short} run with {low} hardware queues per process (< {need}: HIP was "
                  f"initialised before the package could raise GPU_MAX_HW_QUEUES)")
    elif asked:
        reason = f"GJ_ONE_COMM=1 on rank(s) {asked}"
    else:
        reason = ""
    return {"one_comm": bool(short or asked), "hw_queues": low, "reason": reason}


def _raise_file_status(st: int, path, what: str = "") -> None:
    if st == 3:
        raise FileNotFoundError(f"cannot open{what} {path}")
    if st == 4:
        raise ValueError(f"cannot read{what} {path}")
    if st != 0:
        raise RuntimeError(f"unknown error {st} in {path}")


class DistributedGaussJordan:
    """Block-row-cyclic Gauss-Jordan inversion with one rank per process.

    Typical GPU use (under ``torchrun``)::

        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        gj = DistributedGaussJordan(n=32768, m=128)
        gj.generate("random", seed=0)
        stats = gj.solve()                    # collective
        res = gj.residual_generated("random", 0)
    """

    def __init__(self, n: int, m: int, dtype: str = "fp64", chunk_cols: int = 0, eps: float = 1e-15,
                 sync_debug: bool = False, host_threads: int = 0, local_rank: Optional[int] = None,
                 depth: int = 0, pivot: str = "block-min-inv-norm", comm_timeout: float = 600.0):
        C = load_native()
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.backend = dist.get_backend()
        self.n, self.m, self.dtype = int(n), int(m), dtype
        self.comm_mode = {"one_comm": False, "hw_queues": None, "reason": ""}
        if self.backend == "nccl":
            if local_rank is None:
                local_rank = int(os.environ.get("LOCAL_RANK", torch.cuda.current_device()))
            self.local_rank = local_rank
            self.device = C.hip_device(local_rank)
            if self.world > 1:
                # every rank takes the same communicator schedule, before any communicator exists
                self.comm_mode = agree_comm_mode()
                obj = [[C.rccl_unique_id(), C.rccl_unique_id()] if self.rank == 0 else None]
                dist.broadcast_object_list(obj, src=0)
                self.comm = C.rccl_comm(obj[0], self.world, self.rank, local_rank,
                                        one_comm=self.comm_mode["one_comm"])
            else:
                self.comm = C.self_comm()
        else:
            self.local_rank = None
            self.device = C.host_device(host_threads)
            self.comm = C.py_comm(TorchDistComm(), self.rank, self.world) if self.world > 1 else C.self_comm()
        # comm_timeout: seconds any wait on a peer may take before every rank fails with the step,
        # phase and collective it was in (Engine::solve), instead of hanging
        self.engine = C.Engine(self.device, self.comm, self.n, self.m, dtype, chunk_cols, eps, sync_debug, depth,
                               comm_timeout_s=float(comm_timeout), pivot=pivot)
        self.layout = Layout(self.n, self.m, self.world, self.rank)
        self._rows = global_rows(self.n, self.m, self.world, self.rank)

    # ---- input
    def generate(self, kind: str = "absdiff", seed: int = 0) -> None:
        self.engine.generate(kind, int(seed))

    def load(self, A: np.ndarray) -> None:
        """Load this rank's rows of the full matrix A (every rank may pass the full matrix)."""
        A = np.asarray(A, dtype=np.float64)
        self.engine.upload_local_rows(np.ascontiguousarray(A[self._rows]))

    def load_file(self, path: str, nthreads: int = 0) -> None:
        """Collective: every rank maps the file and parses only its own block rows (text in the
        scanf("%lf") accept set, or raw fp64 ``.bin``), so no rank ever holds more than its share of
        the matrix.  Raises ``FileNotFoundError("cannot open ...")`` / ``ValueError("cannot read
        ...")`` on EVERY rank when any rank fails (reference read_matrix, main.cpp:209-282)."""
        st = self.engine.load_file(str(path), int(nthreads))
        _raise_file_status(st, path)

    def residual_file(self, path: str, nthreads: int = 0) -> float:
        """||A inv(A) - I||_inf with A re-read from the file (reference main.cpp:463-519)."""
        st, res = self.engine.residual_file(str(path), int(nthreads))
        _raise_file_status(st, path, " for residual")
        return res

    def load_local_rows(self, rows: np.ndarray) -> None:
        self.engine.upload_local_rows(np.ascontiguousarray(rows, dtype=np.float64))

    # ---- solve
    def solve(self) -> dict:
        return self.engine.solve()

    # ---- output
    def local_rows(self) -> np.ndarray:
        return self.engine.download_local_rows()

    def global_row_ids(self) -> np.ndarray:
        return self._rows

    def gather_inverse(self) -> Optional[np.ndarray]:
        """Full inverse on rank 0 (None elsewhere); host traffic, meant for tests / small n."""
        mine = torch.from_numpy(self.local_rows())
        if self.world == 1:
            return mine.numpy()
        parts = [None] * self.world if self.rank == 0 else None
        dist.gather_object((self._rows, mine.numpy()), parts, dst=0)
        if self.rank != 0:
            return None
        out = np.zeros((self.n, self.n))
        for rows, vals in parts:
            out[rows] = vals
        return out

    def corner(self, nm: int = 10, which: str = "result") -> np.ndarray:
        return self.engine.corner(nm, 1 if which == "result" else 0)

    def residual_generated(self, kind: str = "absdiff", seed: int = 0) -> float:
        return self.engine.residual_generated(kind, int(seed))

    def residual(self, A: np.ndarray) -> float:
        A = np.asarray(A, dtype=np.float64)
        return self.engine.residual_rows(np.ascontiguousarray(A[self._rows]))
