"""HIP runtime settings the engine depends on, applied before the first HIP call of the process.

* ``GPU_MAX_HW_QUEUES`` >= 16.  One process drives the engine's three streams (MAIN, SIDE,
  COMM), torch's stream and, per RCCL communicator, RCCL's internal streams.  Streams beyond the
  HIP queue limit (default 4) SHARE a hardware queue, and a hardware queue executes in order.  The
  engine's progress argument for its two concurrently active RCCL communicators (SIDE: pivot
  records and panel pieces; COMM: row segments) needs their kernels on different queues: an RCCL
  kernel spinning on a peer must never hold back, behind it in the same queue, the other
  communicator's kernel that the peer is waiting for (a cross-rank cycle).  The other condition,
  free compute units for every channel workgroup, holds because the trailing-update workgroups
  never wait on communication and retire within ~1 ms, and 2 communicators x at most 64 channel
  workgroups < 256 CUs.  README.md, "Progress of the two communicators".
* ``HIP_FORCE_DEV_KERNARG=1``: kernel arguments in device memory (measured: =0 costs 3.4 % at
  N = 8192, profiles/small_n_sweep.md).
* ``HSA_ENABLE_IPC_MODE_LEGACY=0`` unless set: RCCL's inter-process buffers between the rank
  processes of one node go through dma-buf IPC (the legacy IPC handles are not supported by the
  drivers this is deployed on: ``hipIpcGetMemHandle: invalid argument``).

Values already set higher are kept; nothing is ever lowered or raised above 32.

HIP reads ``GPU_MAX_HW_QUEUES`` once, when it initialises.  A program that initialised HIP before
importing this package (a torch CUDA call, ``init_process_group(..., device_id=...)``) runs with
whatever was set then, so the value the process really has is recorded here
(:func:`effective_hw_queues`), and when any rank of a multi-rank RCCL job has fewer than 16, EVERY
rank takes the one-communicator schedule (``parallel.dist.agree_comm_mode``; reference: the
collective agreement of main.cpp:371-381) instead of running two communicators on shared queues.
"""
from __future__ import annotations

import os
import sys

MIN_HW_QUEUES = 16
_EFFECTIVE = None  # hardware queues of this process, fixed at the first configure_runtime_env()


def _hip_initialised() -> bool:
    torch = sys.modules.get("torch")
    if torch is None:
        return False
    try:
        return bool(torch.cuda.is_initialized())
    except Exception:
        return False


def effective_hw_queues(rank: int = 0) -> int:
    """Hardware queues per process HIP runs with (or will run with) in this process.
    ``GJ_TEST_HW_QUEUES`` = ``<count>`` or ``<rank>:<count>[,...]`` fakes it (tests)."""
    fake = os.environ.get("GJ_TEST_HW_QUEUES", "")
    for item in filter(None, fake.split(",")):
        r, _, c = item.rpartition(":")
        if not r or int(r) == rank:
            return int(c)
    if _EFFECTIVE is not None:
        return _EFFECTIVE
    try:
        return int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        return 4


def configure_runtime_env(environ=None) -> dict:
    global _EFFECTIVE
    env = os.environ if environ is None else environ
    try:
        cur = int(env.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        cur = 4
    started = environ is None and _hip_initialised()  # too late to change what HIP uses
    if cur < MIN_HW_QUEUES and env.get("GJ_KEEP_HW_QUEUES", "0") != "1":  # (A/B measurements only)
        env["GPU_MAX_HW_QUEUES"] = str(MIN_HW_QUEUES)
    if environ is None and _EFFECTIVE is None:
        _EFFECTIVE = cur if started else int(env["GPU_MAX_HW_QUEUES"])
    env.setdefault("HIP_FORCE_DEV_KERNARG", "1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return {"GPU_MAX_HW_QUEUES": env["GPU_MAX_HW_QUEUES"], "HIP_FORCE_DEV_KERNARG": env["HIP_FORCE_DEV_KERNARG"]}
