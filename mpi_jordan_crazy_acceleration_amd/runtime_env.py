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
"""
from __future__ import annotations

import os

MIN_HW_QUEUES = 16


def configure_runtime_env(environ=None) -> dict:
    env = os.environ if environ is None else environ
    try:
        cur = int(env.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        cur = 4
    if cur < MIN_HW_QUEUES and env.get("GJ_KEEP_HW_QUEUES", "0") != "1":  # (A/B measurements only)
        env["GPU_MAX_HW_QUEUES"] = str(MIN_HW_QUEUES)
    env.setdefault("HIP_FORCE_DEV_KERNARG", "1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return {"GPU_MAX_HW_QUEUES": env["GPU_MAX_HW_QUEUES"], "HIP_FORCE_DEV_KERNARG": env["HIP_FORCE_DEV_KERNARG"]}
