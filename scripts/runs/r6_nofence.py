#!/usr/bin/env python3
"""Round 6: the round-5 no-fence failure (GJ_EVENT_RELEASE=none: residual 600 in
test_golden_residuals.py::test_n2048_p8_gpu_async_ranks[30]) run ONCE per depth with GJ_VERIFY=1,
so the consumption-point and rank-local hand-over hashes name the edge (profiles/verify_r6.md).
Run with GJ_EVENT_RELEASE=none GJ_VERIFY=1 in the environment."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import mpi_jordan_crazy_acceleration_amd as gj  # noqa: E402

for depth in (2, 4):
    rep = gj.GaussJordan(block_size=30, ranks=8, device="gpu", comm="async", jitter_us=20.0, depth=depth).run(
        2048, gen="absdiff")
    print(json.dumps({"depth": depth, "status": rep["status"], "residual": rep.get("residual"),
                      "message": rep.get("message"), "env": {k: v for k, v in os.environ.items()
                                                              if k.startswith("GJ_")}}), flush=True)
