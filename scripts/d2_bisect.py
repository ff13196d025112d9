"""Reproduce the golden-residual test's order (n = 8192, m = 60, p = 2, 4, 8 in one process) (temporary)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpi_jordan_crazy_acceleration_amd as gj  # noqa: E402

for p in (2, 4, 8, 8, 2, 8):
    g = gj.GaussJordan(block_size=60, ranks=p, device="gpu", comm="async")
    rep = g.run(8192, gen="absdiff")
    print("p", p, rep["status"], rep["residual"], rep.get("policy", {}).get("depth") if isinstance(rep.get("policy"), dict) else "", flush=True)
