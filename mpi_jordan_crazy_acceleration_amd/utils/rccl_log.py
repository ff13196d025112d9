"""Which transport RCCL connected the ranks with (xGMI peer-to-peer vs sockets), from its own log.

RCCL picks a transport per channel connection when a communicator first uses it and logs it at
``NCCL_DEBUG=INFO`` (``Channel 00/0 : 0[0] -> 1[1] via P2P/IPC ...``).  ``bench.py`` points
``NCCL_DEBUG_FILE`` at a per-rank file before the first RCCL call and reports the counts per
transport in its JSON line (``rccl_transport``), so a scaling record says what the collectives
actually ran over: ``P2P/...`` (xGMI peer-to-peer on one node), ``SHM``, or ``NET/Socket`` (the
one-GPU ``--same-gpu`` rehearsal)."""
from __future__ import annotations

import os
import re
from collections import Counter
from typing import Optional

_VIA = re.compile(r"Channel \d+/\d+ ?: .*?\bvia\s+([A-Za-z0-9_]+(?:/[A-Za-z0-9_]+)?)")


def enable(path: str, environ=None) -> Optional[str]:
    """Route RCCL's INFO log of the connection setup to a file; returns the file to parse (None:
    the user already sends an INFO log to a file of their own naming, which is left alone).  A
    quieter NCCL_DEBUG (WARN, as images often set) is raised to INFO for this process: the
    connection lines are only logged at INFO.  Must run before the process's first RCCL call."""
    env = os.environ if environ is None else environ
    level = env.get("NCCL_DEBUG", "").upper()
    if level in ("INFO", "TRACE") and env.get("NCCL_DEBUG_FILE"):
        return None
    if level not in ("INFO", "TRACE"):
        env["NCCL_DEBUG"] = "INFO"
        env["NCCL_DEBUG_SUBSYS"] = "INIT,P2P,NET"
    env["NCCL_DEBUG_FILE"] = path
    return path


def transports(path: Optional[str]) -> Optional[dict]:
    """{transport: channel connections} found in an RCCL log (None: no log)."""
    if not path or not os.path.exists(path):
        return None
    seen = Counter()
    with open(path, errors="replace") as f:
        for line in f:
            m = _VIA.search(line)
            if m:
                seen[m.group(1)] += 1
    return dict(seen)
