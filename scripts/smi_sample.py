#!/usr/bin/env python3
"""Sample the GPU's shader clock, power and temperature while another command runs.

    python3 scripts/smi_sample.py OUT.jsonl -- python3 bench.py --steps 20 --warmup 5

Starts the command as a child process (this script never touches the GPU itself), and every
``--interval`` seconds until the child exits appends one line ``{"t": seconds since start, "raw":
<amd-smi metric --json output>}`` to OUT.jsonl (``rocm-smi --json`` if amd-smi is unavailable).
The child's exit status is returned.  ``scripts/smi_summary.py`` reduces the samples to
per-interval clock / power tables (profiles/sustained_r6.md).
"""
from __future__ import annotations

import json
import subprocess
import sys
import time


def _query(cmd):
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=10)
    except Exception as e:  # noqa: BLE001 -- a failed sample is recorded, not fatal
        return None, str(e)
    if r.returncode != 0:
        return None, (r.stderr or r.stdout)[-500:]
    try:
        return json.loads(r.stdout), None
    except ValueError:
        return None, r.stdout[-500:]


def main(argv):
    interval = 0.5
    if "--interval" in argv:
        i = argv.index("--interval")
        interval = float(argv[i + 1])
        del argv[i:i + 2]
    out, sep, cmd = argv[0], argv[1], argv[2:]
    assert sep == "--" and cmd, __doc__
    queries = [["amd-smi", "metric", "--power", "--clock", "--temperature", "--usage", "--json"],
               ["amd-smi", "metric", "--json"],
               ["rocm-smi", "--showclocks", "--showpower", "--showtemp", "--showuse", "--json"]]
    child = subprocess.Popen(cmd)
    t0 = time.monotonic()
    q = None
    with open(out, "w") as f:
        while child.poll() is None:
            ts = time.monotonic() - t0
            raw = err = None
            for cand in ([q] if q else queries):
                raw, err = _query(cand)
                if raw is not None:
                    q = cand
                    break
            f.write(json.dumps({"t": round(ts, 3), "cmd": q[0:2] if q else None, "raw": raw, "err": err}) + "\n")
            f.flush()
            time.sleep(max(0.0, interval - (time.monotonic() - t0 - ts)))
    return child.wait()


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
